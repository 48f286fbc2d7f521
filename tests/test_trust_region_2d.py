"""CPU: the trust-region 2-D subproblem of optim_points' trf driver (mq_trust_region_2d, host code of
csrc/optim_trf.hip) against the numpy restatement oracle/trf.py:solve_trust_region_2d (scipy 1.15.3
optimize/_lsq/common.py, pinned to scipy by tests/test_oracle_trf.py).  No HIP call is made.

The library finds the quartic's real roots by bracketing and bisection instead of np.roots' companion
eigenvalues, so boundary steps agree to rounding (1e-9 relative), interior (Newton) steps bit for bit in
practice; the degenerate case scipy cannot solve (no real root: np.argmin over nothing raises) returns a point on
the boundary no worse than the Cauchy point."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd")]


@pytest.fixture(scope="module")
def lib():
    from mqhip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmq_hip.so not built")
    return _lib.load()


def _solve(lib, B, g, Delta):
    Bv = np.array([B[0, 0], B[0, 1], B[1, 1]], np.float64)
    gv = np.asarray(g, np.float64)
    p = np.zeros(2, np.float64)
    rc = lib.mq_trust_region_2d(C.c_void_p(Bv.ctypes.data), C.c_void_p(gv.ctypes.data), float(Delta),
                                C.c_void_p(p.ctypes.data))
    assert rc == 0
    return p


def _q(B, g, p):
    return 0.5 * p @ B @ p + g @ p


def test_trust_region_2d_matches_numpy_restatement(lib):
    from oracle.trf import solve_trust_region_2d
    rng = np.random.default_rng(5)
    n_int = n_bnd = 0
    for _ in range(400):
        A = rng.standard_normal((2, 2))
        B = A @ A.T if rng.random() < 0.6 else (A + A.T) / 2     # positive definite or indefinite
        g = rng.standard_normal(2) * 10 ** rng.uniform(-2, 2)
        Delta = 10 ** rng.uniform(-2, 1)
        p_ref, newton = solve_trust_region_2d(B, g, Delta)
        p = _solve(lib, B, g, Delta)
        if newton:
            n_int += 1
            np.testing.assert_allclose(p, p_ref, rtol=1e-12, atol=1e-15)
        else:
            n_bnd += 1
            assert abs(np.linalg.norm(p) - Delta) <= 1e-9 * Delta
            # the same boundary minimiser (or, where two roots tie, an equally good one)
            assert _q(B, g, p) <= _q(B, g, p_ref) + 1e-9 * (abs(_q(B, g, p_ref)) + 1e-12)
            np.testing.assert_allclose(p, p_ref, rtol=1e-6, atol=1e-9 * Delta)
    assert n_int > 50 and n_bnd > 50


def test_trust_region_2d_degenerate_returns_boundary_point(lib):
    """B = 0, g = 0: the quartic is identically zero after scaling (no sign change, no root), where scipy's argmin
    raises.  The library still returns a point on the trust-region boundary."""
    B = np.zeros((2, 2))
    g = np.zeros(2)
    p = _solve(lib, B, g, 2.0)
    assert np.isfinite(p).all() and abs(np.linalg.norm(p) - 2.0) < 1e-12
    # a negative-definite B with g = 0: every boundary point is optimal; the answer lies on the boundary
    p = _solve(lib, -np.eye(2), np.zeros(2), 0.5)
    assert abs(np.linalg.norm(p) - 0.5) < 1e-12


def test_trust_region_2d_rejects_bad_arguments(lib):
    z = np.zeros(3)
    assert lib.mq_trust_region_2d(None, None, 1.0, None) == -1
    assert lib.mq_trust_region_2d(C.c_void_p(z.ctypes.data), C.c_void_p(z.ctypes.data), 0.0,
                                  C.c_void_p(z.ctypes.data)) == -2
    assert lib.mq_trust_region_2d(C.c_void_p(z.ctypes.data), C.c_void_p(z.ctypes.data), float("nan"),
                                  C.c_void_p(z.ctypes.data)) == -2
