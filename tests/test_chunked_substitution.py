"""CPU: the chunked block-banded substitution that optim_precond_lds_kernel runs (csrc/optim.hip), as
a numpy model, against the plain sequential substitution.

The preconditioner solves L y = u (forward) and L^T z = v (backward) for a block lower-triangular L
with 3x3 blocks and bandwidth n (one joint series of optim_points, cameras.py:1116-1190).  The kernel
cuts the F frames into K = opt_chunks(F, n) chunks [c F / K, (c + 1) F / K), solves every chunk with
zero incoming vectors at once, then stitches: the true incoming vectors of chunk c are the last n
results of chunk c - 1 corrected by the chunk responses G (computed once per factorisation), and
every frame adds G_f S_c.  This model follows those steps and must reproduce the sequential solve to
rounding.  No GPU is used."""
import numpy as np
import pytest


def opt_chunks(F, n):
    """csrc/optim.hip opt_chunks: ~sqrt(F), at most 16, every chunk at least n frames."""
    k = 1
    while (k + 1) * (k + 1) <= F:
        k += 1
    k = min(k, 16)
    k = min(k, F // max(n, 1))
    return max(k, 1)


def sequential_forward(M, u):
    """y_f = u_f - sum_d M[f, d-1] y_{f-d} (M[f, d-1] = 0 where f - d < 0)."""
    F, n = M.shape[:2]
    y = np.zeros_like(u)
    for f in range(F):
        acc = u[f].copy()
        for d in range(n, 0, -1):
            if f - d >= 0:
                acc -= M[f, d - 1] @ y[f - d]
        y[f] = acc
    return y


def chunk_responses(M, a, e, n):
    """G[f, k-1] (f in [a, e)): the response of frame f to a unit incoming vector at frame a - k."""
    G = np.zeros((e - a, n, 3, 3))
    for k in range(1, n + 1):
        for comp in range(3):
            hist = {a - d: np.zeros(3) for d in range(1, n + 1)}
            hist[a - k] = np.eye(3)[comp]
            for f in range(a, e):
                g = np.zeros(3)
                for d in range(n, 0, -1):
                    g -= M[f, d - 1] @ hist[f - d]
                hist[f] = g
                G[f - a, k - 1][:, comp] = g
    return G


def chunked_forward(M, u):
    F, n = M.shape[:2]
    K = opt_chunks(F, n)
    bounds = [c * F // K for c in range(K + 1)]
    # phase 1: every chunk with zero incoming vectors
    yh = np.zeros_like(u)
    for c in range(K):
        a, e = bounds[c], bounds[c + 1]
        Mc = M[a:e].copy()
        for f in range(e - a):                      # drop the terms reaching before the chunk
            for d in range(1, n + 1):
                if f - d < 0:
                    Mc[f, d - 1] = 0.0
        yh[a:e] = sequential_forward(Mc, u[a:e])
    Gs = [None] + [chunk_responses(M, bounds[c], bounds[c + 1], n) for c in range(1, K)]
    # phase 2: the true incoming vectors, chunk by chunk
    S = [None] * K
    for c in range(1, K):
        a = bounds[c]
        Sc = np.zeros((n, 3))
        for k in range(1, n + 1):
            g = a - k                                # a frame of chunk c - 1
            v = yh[g].copy()
            if c >= 2:
                Gg = Gs[c - 1][g - bounds[c - 1]]
                for j in range(n):
                    v += Gg[j] @ S[c - 1][j]
            Sc[k - 1] = v
        S[c] = Sc
    # phase 3: every frame
    y = yh.copy()
    for c in range(1, K):
        a, e = bounds[c], bounds[c + 1]
        for f in range(a, e):
            for k in range(n):
                y[f] += Gs[c][f - a, k] @ S[c][k]
    return y, K


@pytest.mark.parametrize("F,n", [(300, 2), (37, 1), (64, 3), (9, 2), (2, 1), (513, 2)])
def test_chunked_forward_equals_sequential(F, n):
    rng = np.random.default_rng(F * 10 + n)
    # M blocks of a well-conditioned banded factor (|M| < 1 keeps the responses bounded, as the
    # pre-multiplied Cholesky blocks of an SPD band matrix are)
    M = rng.normal(0, 0.25 / n, (F, n, 3, 3))
    for f in range(F):
        for d in range(1, n + 1):
            if f - d < 0:
                M[f, d - 1] = 0.0
    u = rng.normal(0, 1, (F, 3))
    ref = sequential_forward(M, u)
    got, K = chunked_forward(M, u)
    assert K == opt_chunks(F, n)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-10 * np.abs(ref).max())


def test_opt_chunks_bounds():
    assert opt_chunks(300, 2) == 16
    assert opt_chunks(37, 1) == 6
    assert opt_chunks(2, 1) == 1
    for F in range(1, 600, 7):
        for n in (1, 2, 3):
            K = opt_chunks(F, n)
            lens = [(c + 1) * F // K - c * F // K for c in range(K)]
            assert 1 <= K <= 16 and min(lens) >= min(n, F) and max(lens) - min(lens) <= 1
