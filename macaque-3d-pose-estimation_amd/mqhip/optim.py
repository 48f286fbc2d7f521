"""CameraGroup.optim_points on the GPU (row a16).

Host side of ``mq_optim_points``: the parameter initialisation the reference runs
before its solver (cameras.py:1116-1150 -- NaN interpolation per series, a
7-frame median filter to set the smoothness scale, joint-length medians with
the MAD outlier rule of _initialize_params_triangulation :1670-1697) is O(F*J)
bookkeeping done here in numpy; the solve (every residual, Jacobian and linear
step) runs in libmq_hip.  There is no CPU solver behind this module.

``optim_points_batch`` refines several animals in one call (they are
independent problems sharing the cameras).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

LOSSES = {"linear": 0, "soft_l1": 1, "huber": 2}


def interpolate_series(vals):
    """cameras.py:135-145: linear fill of NaNs along one series (all-NaN -> 0)."""
    nans = np.isnan(vals)
    out = np.array(vals, dtype=np.float64, copy=True)
    good = ~nans
    if not good.any():
        out[:] = 0
        return out
    out[nans] = np.interp(np.flatnonzero(nans), np.flatnonzero(good), vals[good])
    return out


def median_filter_series(values, size=7):
    """cameras.py:129-133: reflect-pad by size+5, zero-padded running median, crop."""
    pad = size + 5
    v = np.pad(values, (pad, pad), mode="reflect")
    h = size // 2
    vz = np.pad(v, (h, h), mode="constant")
    win = np.lib.stride_tricks.sliding_window_view(vz, size)
    return np.median(win, axis=-1)[pad:-pad]


def median_filter_columns(values, size=7):
    """median_filter_series on every column of values (F, n) at once: the same padding, windows and
    medians (np.median of the same 7 values), so the same numbers."""
    pad = size + 5
    v = np.pad(values, ((pad, pad), (0, 0)), mode="reflect")
    h = size // 2
    vz = np.pad(v, ((h, h), (0, 0)), mode="constant")
    win = np.lib.stride_tricks.sliding_window_view(vz, size, axis=0)[pad:-pad]   # (F, n, size)
    if size % 2 and not np.isnan(vz).any():
        # odd window without NaN: np.median is the middle order statistic, exactly
        return np.sort(win, axis=-1)[..., size // 2]
    return np.median(win, axis=-1)


def smooth_scale(p3ds_intp, scale_smooth):
    """scale_smooth_full = scale_smooth / mean|diff(medfilt7(interp p3d))| (cameras.py:1133-1137)."""
    F = p3ds_intp.shape[0]
    med = median_filter_columns(p3ds_intp.reshape(F, -1), 7).reshape(p3ds_intp.shape)
    # np.mean's summation order follows the memory layout: lay med out as the reference's
    # np.apply_along_axis(medfilt_data, 0, ...) result is laid out (frames fastest)
    buf = np.empty(p3ds_intp.shape[1:] + (F,), dtype=np.float64)
    buf[...] = np.moveaxis(med, 0, -1)
    med = np.moveaxis(buf, -1, 0)
    return scale_smooth * (1.0 / np.mean(np.abs(np.diff(med, axis=0))))


def initial_lengths(p3ds_intp, constraints, constraints_weak):
    """_initialize_params_triangulation (cameras.py:1670-1697): median limb lengths, 0 / outlier -> median."""
    def med_len(pairs):
        pairs = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
        if len(pairs) == 0:
            return np.zeros(0, dtype=np.float64)
        # every pair's per-frame length at once (F, P), then each column's median
        d = np.linalg.norm(p3ds_intp[:, pairs[:, 0]] - p3ds_intp[:, pairs[:, 1]], axis=2)
        return np.median(d, axis=0).astype(np.float64)
    jl, jlw = med_len(constraints), med_len(constraints_weak)
    alll = np.hstack([jl, jlw])
    if alll.size == 0:
        return jl, jlw
    med = np.median(alll)
    if med == 0:
        med = 1e-3
    mad = np.median(np.abs(alll - med))
    for arr in (jl, jlw):
        arr[arr == 0] = med
        arr[arr > med + mad * 5] = med
    return jl, jlw


def prepare(p3ds, constraints, constraints_weak, scale_smooth):
    """x0 and scale_smooth_full for one animal, exactly as the reference builds them."""
    p3ds = np.asarray(p3ds, dtype=np.float64)
    F, J, _ = p3ds.shape
    intp = p3ds.copy()
    flat = intp.reshape(F, -1)
    for i in np.flatnonzero(np.isnan(flat).any(axis=0)):   # only the series with gaps (others unchanged)
        flat[:, i] = interpolate_series(flat[:, i])
    ssf = smooth_scale(intp, scale_smooth)
    jl, jlw = initial_lengths(intp, constraints, constraints_weak)
    x0 = np.hstack([intp.ravel(), jl, jlw])
    x0[~np.isfinite(x0)] = 0
    return x0, ssf


def _pairs(c):
    c = np.asarray(c, dtype=np.int32).reshape(-1, 2) if len(c) else np.zeros((0, 2), np.int32)
    return c


def optim_points_batch(cgroup, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4, scale_length=2,
                       scale_length_weak=0.5, reproj_error_threshold=15, reproj_loss="soft_l1", n_deriv_smooth=1,
                       joint_len=None, max_iter=200, ftol=1e-3, verbose=False, return_stats=False):
    """points (B,C,F,J,2) with NaN for missing, p3ds (B,F,J,3) initial triangulation.

    joint_len=None: lengths are optimised (optim_points); a (n_strong+n_weak,) array fixes
    them (optim_points_jointlenfix, cameras.py:1192-1415).
    Returns p3ds_new (B,F,J,3) and joint_len (B, n_strong+n_weak)."""
    points = np.asarray(points, dtype=np.float64)
    p3ds = np.asarray(p3ds, dtype=np.float64)
    B, C, F, J, _ = points.shape
    assert C == len(cgroup.cameras), (
        "Invalid points shape, first dim should be equal to number of cameras ({}), but shape is {}".format(
            len(cgroup.cameras), points.shape[1:]))
    assert p3ds.shape == (B, F, J, 3)
    if reproj_loss not in LOSSES:
        raise ValueError(f"unknown reproj_loss {reproj_loss!r}")
    cons, consw = _pairs(constraints), _pairs(constraints_weak)
    nS, nW = len(cons), len(consw)
    xs, ssf = [], []
    for b in range(B):
        x0, s = prepare(p3ds[b], cons, consw, scale_smooth)
        if joint_len is not None:
            x0[F * J * 3:] = np.asarray(joint_len, dtype=np.float64).ravel()
        xs.append(x0)
        ssf.append(s)
    dev = cgroup._dev()
    ctx = cgroup._ctx()
    x_d = torch.from_numpy(np.stack(xs)).to(dev)
    p2_d = torch.from_numpy(np.ascontiguousarray(points)).to(dev)
    cams = cgroup.cams_tensor()
    allc = np.ascontiguousarray(np.vstack([cons, consw]).astype(np.int32)) if nS + nW else np.zeros((1, 2), np.int32)
    ssf_h = np.ascontiguousarray(np.array(ssf, dtype=np.float64))
    stats = np.zeros((B, 4), dtype=np.float64)
    import ctypes
    rc = ctx.lib.mq_optim_points(
        ctx.handle, _lib.ptr(cams), C, _lib.ptr(p2_d), _lib.ptr(x_d), B, F, J,
        allc.ctypes.data_as(ctypes.c_void_p), nS, nW, ssf_h.ctypes.data_as(ctypes.c_void_p),
        float(scale_length), float(scale_length_weak), float(reproj_error_threshold), LOSSES[reproj_loss],
        int(n_deriv_smooth), 0 if joint_len is None else 1, int(max_iter), float(ftol),
        stats.ctypes.data_as(ctypes.c_void_p), _lib.stream_ptr(dev))
    _lib.check(rc, "mq_optim_points")
    x = x_d.cpu().numpy()
    if verbose:
        for b in range(B):
            print(f"optim_points[{b}]: cost {stats[b, 0]:.6g} -> {stats[b, 1]:.6g} in {int(stats[b, 2])} LM steps")
    out = x[:, :F * J * 3].reshape(B, F, J, 3), x[:, F * J * 3:]
    if return_stats:
        return out + (stats, np.array(ssf))
    return out


def optim_points_gpu(cgroup, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4, scale_length=2,
                     scale_length_weak=0.5, reproj_error_threshold=15, reproj_loss="soft_l1", n_deriv_smooth=1,
                     scores=None, verbose=False, joint_len=None, max_iter=200, ftol=1e-3):
    """CameraGroup.optim_points signature (cameras.py:1116): points (C,F,J,2), p3ds (F,J,3)
    -> (p3ds_new (F,J,3), joint_len (n_strong + n_weak,))."""
    if scores is not None:
        raise NotImplementedError("score-weighted reprojection is disabled on the reference path (step4:252)")
    p3, jl = optim_points_batch(cgroup, np.asarray(points)[None], np.asarray(p3ds)[None], constraints,
                                constraints_weak, scale_smooth, scale_length, scale_length_weak,
                                reproj_error_threshold, reproj_loss, n_deriv_smooth, joint_len=joint_len,
                                max_iter=max_iter, ftol=ftol, verbose=verbose)
    return p3[0], jl[0]
