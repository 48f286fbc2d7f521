"""CPU: mq_optim_prepare -- optim_points' parameter initialisation in libmq_hip's host code -- equals the
oracle's restatement of cameras.py:1116-1150 / 1670-1697 (np.interp gap filling, medfilt_data with
scipy's medfilt, np.median limb lengths with the MAD rule, np.mean of |diff|) BIT FOR BIT: x0 and
scale_smooth_full, over gaps at the start / middle / end, all-NaN series, short clips (reflect padding
wider than the clip) and clips longer than numpy's 8192-element reduction buffer.  No HIP call is made
(host pointers only), so this runs without a GPU."""
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    from mqhip import _lib
    return _lib.load()


def _cons():
    from mqhip import synth
    return (np.asarray(synth.constraint_indices(synth.CONSTRAINTS), np.int32).reshape(-1, 2),
            np.asarray(synth.constraint_indices(synth.CONSTRAINTS_WEAK), np.int32).reshape(-1, 2))


def _prepare(lib, p3ds, cons, weak, scale_smooth):
    B, F, J, _ = p3ds.shape
    allc = np.ascontiguousarray(np.vstack([cons, weak]).astype(np.int32))
    nx = F * J * 3 + len(cons) + len(weak)
    x0 = np.zeros((B, nx))
    ssf = np.zeros(B)
    p = np.ascontiguousarray(p3ds, dtype=np.float64)
    rc = lib.mq_optim_prepare(p.ctypes.data_as(ctypes.c_void_p), B, F, J, allc.ctypes.data_as(ctypes.c_void_p),
                              len(cons), len(weak), float(scale_smooth), x0.ctypes.data_as(ctypes.c_void_p),
                              ssf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, lib.mq_last_error()
    return x0, ssf


def _clip(F, seed, gaps=True):
    from mqhip import synth
    rng = np.random.default_rng(seed)
    p = synth.make_skeletons(2, F, seed=seed) + rng.normal(0, 3.0, (2, F, 17, 3))
    if gaps:
        for a in range(2):
            for _ in range(max(1, F // 10)):
                j, f0 = rng.integers(0, 17), rng.integers(0, F)
                p[a, f0:f0 + rng.integers(1, 12), j] = np.nan
            p[a, :rng.integers(1, 4), 3] = np.nan               # leading gap
            p[a, F - rng.integers(1, 4):, 5] = np.nan           # trailing gap
            p[a, :, 7] = np.nan                                 # all-NaN joint
            p[a, rng.integers(0, F), 9, 1] = np.nan              # single-axis gap
    return p


@pytest.mark.parametrize("F,seed", [(300, 0), (24, 1), (5, 2), (13, 3), (480, 4), (1200, 5), (2, 6)])
def test_optim_prepare_equals_oracle_bitwise(lib, F, seed):
    from oracle.geometry import optim_init
    cons, weak = _cons()
    p = _clip(F, seed)
    x0, ssf = _prepare(lib, p, cons, weak, 3)
    for a in range(p.shape[0]):
        rx, rs = optim_init(p[a].copy(), cons, weak, 3)
        assert x0[a].tobytes() == rx.tobytes(), np.flatnonzero(x0[a] != rx)[:10]
        assert np.float64(ssf[a]).tobytes() == np.float64(rs).tobytes(), (ssf[a], rs)


def test_optim_prepare_without_gaps_and_with_outlier_lengths(lib):
    from oracle.geometry import optim_init
    cons, weak = _cons()
    p = _clip(300, 9, gaps=False)
    p[1, :, 4] = p[1, :, 0]             # zero-length limb (nose, right_ear) -> median
    p[1, :, 16] += 5000.0               # far outlier limb -> median
    x0, ssf = _prepare(lib, p, cons, weak, 3)
    for a in range(2):
        rx, rs = optim_init(p[a].copy(), cons, weak, 3)
        assert x0[a].tobytes() == rx.tobytes()
        assert ssf[a] == rs


def test_optim_prepare_rejects_bad_arguments(lib):
    x = np.zeros(10)
    c = np.array([[0, 99]], np.int32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert lib.mq_optim_prepare(vp(x), 1, 2, 17, vp(c), 1, 0, 3.0, vp(x), vp(x)) == -2
    assert lib.mq_optim_prepare(None, 1, 2, 17, vp(c), 0, 0, 3.0, vp(x), vp(x)) == -1
