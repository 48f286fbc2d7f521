"""CameraGroup.optim_points on the GPU (row a16).

Host side of ``mq_optim_points``: the parameter initialisation the reference runs
before its solver (cameras.py:1116-1150 -- NaN interpolation per series, a
7-frame median filter to set the smoothness scale, joint-length medians with
the MAD outlier rule of _initialize_params_triangulation :1670-1697) is libmq_hip's
host C++ ``mq_optim_prepare`` (numpy's rounding and summation orders, one thread per
animal); the solve (every residual, Jacobian and linear step) runs in libmq_hip's
kernels.  There is no CPU solver behind this module.

Two solvers (ABI 7):
  "trf" (default) -- the reference's own algorithm, scipy's least_squares(method='trf') with lsmr trust-region
          steps (cameras.py:1166-1180; scipy 1.15.3 trf_no_bounds), restated on the GPU
          (csrc/optim_trf.hip): the parity mode, it stops where scipy stops;
  "lm"   -- Levenberg-Marquardt + PCG with its own stop rule (csrc/optim.hip): lands closer to the
          converged solution than scipy's ftol-1e-3 stop, in fewer, heavier steps.

``optim_points_batch`` refines several animals in one call (they are
independent problems sharing the cameras).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

LOSSES = {"linear": 0, "soft_l1": 1, "huber": 2}
SOLVERS = {"trf": 0, "lm": 1}
_DEFAULT = {"solver": "trf"}


def set_default_solver(name):
    """Select the solver step 4 and CameraGroup.optim_points use ("trf", the default, or "lm"); returns the
    previous one (bench.py times config 4 with both)."""
    if name not in SOLVERS:
        raise ValueError(f"unknown solver {name!r}")
    prev, _DEFAULT["solver"] = _DEFAULT["solver"], name
    return prev

# Set to a list to record every optim_points_batch call (problem size, LM steps per individual, wall ms):
# the config-3 clip driver (tools/run_clip_sharded.py) reports step 4's solver work from it.
CALL_LOG = None


def prepare_batch(p3ds, constraints, constraints_weak, scale_smooth):
    """x0 (B, F*J*3 + n_strong + n_weak) and scale_smooth_full (B) for every animal, exactly as the
    reference builds them (cameras.py:1116-1150, 1670-1697) -- mq_optim_prepare, libmq_hip host code
    (one thread per animal; bit-exact vs the oracle's numpy restatement, tests/test_optim_host.py)."""
    import ctypes
    p3ds = np.ascontiguousarray(p3ds, dtype=np.float64)
    B, F, J, _ = p3ds.shape
    cons, consw = _pairs(constraints), _pairs(constraints_weak)
    allc = np.ascontiguousarray(np.vstack([cons, consw]).astype(np.int32)) if len(cons) + len(consw) \
        else np.zeros((1, 2), np.int32)
    x0 = np.empty((B, F * J * 3 + len(cons) + len(consw)), dtype=np.float64)
    ssf = np.empty(B, dtype=np.float64)
    lib = _lib.load()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _lib.check(lib.mq_optim_prepare(vp(p3ds), B, F, J, vp(allc), len(cons), len(consw), float(scale_smooth), vp(x0),
                                    vp(ssf)), "mq_optim_prepare")
    return x0, ssf


def _pairs(c):
    c = np.asarray(c, dtype=np.int32).reshape(-1, 2) if len(c) else np.zeros((0, 2), np.int32)
    return c


def optim_points_batch(cgroup, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4, scale_length=2,
                       scale_length_weak=0.5, reproj_error_threshold=15, reproj_loss="soft_l1", n_deriv_smooth=1,
                       joint_len=None, max_iter=200, ftol=1e-3, verbose=False, return_stats=False, solver=None,
                       max_nfev=None):
    """points (B,C,F,J,2) with NaN for missing, p3ds (B,F,J,3) initial triangulation.

    joint_len=None: lengths are optimised (optim_points); a (n_strong+n_weak,) array fixes
    them (optim_points_jointlenfix, cameras.py:1192-1415).
    solver: "trf" (scipy's algorithm; max_nfev as scipy's, None = 100 x parameters) or "lm" (max_iter LM steps);
    None = the module default (set_default_solver).
    Returns p3ds_new (B,F,J,3) and joint_len (B, n_strong+n_weak); with return_stats also the (B, 8) stats
    (initial cost, final cost, iterations, status, nfev, njev, lsmr iterations, longest lsmr run) and
    scale_smooth_full."""
    points = np.asarray(points, dtype=np.float64)
    p3ds = np.asarray(p3ds, dtype=np.float64)
    B, C, F, J, _ = points.shape
    assert C == len(cgroup.cameras), (
        "Invalid points shape, first dim should be equal to number of cameras ({}), but shape is {}".format(
            len(cgroup.cameras), points.shape[1:]))
    assert p3ds.shape == (B, F, J, 3)
    if reproj_loss not in LOSSES:
        raise ValueError(f"unknown reproj_loss {reproj_loss!r}")
    solver = _DEFAULT["solver"] if solver is None else solver
    if solver not in SOLVERS:
        raise ValueError(f"unknown solver {solver!r}")
    limit = (int(max_nfev) if max_nfev else 0) if solver == "trf" else int(max_iter)
    cons, consw = _pairs(constraints), _pairs(constraints_weak)
    nS, nW = len(cons), len(consw)
    xs, ssf = prepare_batch(p3ds, cons, consw, scale_smooth)
    if joint_len is not None:
        xs[:, F * J * 3:] = np.asarray(joint_len, dtype=np.float64).ravel()
    dev = cgroup._dev()
    ctx = cgroup._ctx()
    x_d = torch.from_numpy(xs).to(dev)
    p2_d = torch.from_numpy(np.ascontiguousarray(points)).to(dev)
    cams = cgroup.cams_tensor()
    allc = np.ascontiguousarray(np.vstack([cons, consw]).astype(np.int32)) if nS + nW else np.zeros((1, 2), np.int32)
    ssf_h = np.ascontiguousarray(np.array(ssf, dtype=np.float64))
    stats = np.zeros((B, 8), dtype=np.float64)
    import ctypes
    import time
    t0 = time.perf_counter()
    rc = ctx.lib.mq_optim_points(
        ctx.handle, _lib.ptr(cams), C, _lib.ptr(p2_d), _lib.ptr(x_d), B, F, J,
        allc.ctypes.data_as(ctypes.c_void_p), nS, nW, ssf_h.ctypes.data_as(ctypes.c_void_p),
        float(scale_length), float(scale_length_weak), float(reproj_error_threshold), LOSSES[reproj_loss],
        int(n_deriv_smooth), 0 if joint_len is None else 1, limit, float(ftol), SOLVERS[solver],
        stats.ctypes.data_as(ctypes.c_void_p), _lib.stream_ptr(dev))
    _lib.check(rc, "mq_optim_points")
    x = x_d.cpu().numpy()
    if CALL_LOG is not None:
        CALL_LOG.append({"B": B, "F": F, "J": J, "solver": solver, "iterations": stats[:, 2].astype(int).tolist(),
                         "status": stats[:, 3].astype(int).tolist(), "nfev": stats[:, 4].astype(int).tolist(),
                         "lsmr": stats[:, 6].astype(int).tolist(), "ms": round((time.perf_counter() - t0) * 1e3, 2)})
    if verbose:
        for b in range(B):
            print(f"optim_points[{b}] ({solver}): cost {stats[b, 0]:.6g} -> {stats[b, 1]:.6g} in {int(stats[b, 2])} "
                  f"iterations, status {int(stats[b, 3])}")
    out = x[:, :F * J * 3].reshape(B, F, J, 3), x[:, F * J * 3:]
    if return_stats:
        return out + (stats, ssf)
    return out


def optim_points_gpu(cgroup, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4, scale_length=2,
                     scale_length_weak=0.5, reproj_error_threshold=15, reproj_loss="soft_l1", n_deriv_smooth=1,
                     scores=None, verbose=False, joint_len=None, max_iter=200, ftol=1e-3, max_nfev=None):
    """CameraGroup.optim_points signature (cameras.py:1116): points (C,F,J,2), p3ds (F,J,3)
    -> (p3ds_new (F,J,3), joint_len (n_strong + n_weak,))."""
    if scores is not None:
        raise NotImplementedError("score-weighted reprojection is disabled on the reference path (step4:252)")
    p3, jl = optim_points_batch(cgroup, np.asarray(points)[None], np.asarray(p3ds)[None], constraints,
                                constraints_weak, scale_smooth, scale_length, scale_length_weak,
                                reproj_error_threshold, reproj_loss, n_deriv_smooth, joint_len=joint_len,
                                max_iter=max_iter, ftol=ftol, verbose=verbose, max_nfev=max_nfev)
    return p3[0], jl[0]
