"""GPU optim_points (mq_optim_points) vs the scipy-TRF oracle (row a16), both solvers.

Tolerance: the GPU solution must lie within
max(|scipy(ftol=1e-3) - scipy(ftol=1e-10)| band, 1 mm median / 5 mm p99) of the
scipy result run with the reference's own arguments (cameras.py:1166-1180,
step4:248-258 / config_tmpl.toml:89-97).  The objective is also checked
directly: evaluated by the oracle's residual function, the GPU optimum may not
be worse than scipy's by more than 0.1 %.  The trf solver (the default since ABI 7,
scipy's own algorithm restated) must in addition land within 1 mm (median) / 5 mm (p99)
of scipy's answer itself, with scipy's Jacobian-evaluation count +-1.  Parity is pinned
to the oracle only (scipy least_squares is unpinned by the reference).
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

ARGS = dict(scale_smooth=3, scale_length=5, scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3)


def _problem(F, drop=0.1, gap=False, seed=3):
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(1, F)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=drop, seed=seed)
    o = CameraGroupOracle(cams)
    pts = kp2d[0].transpose(1, 0, 2, 3)
    p2 = pts[..., :2].copy()
    p2[pts[..., 2] < 0.5] = np.nan
    if gap:
        p2[:, F // 3:F // 3 + 8, 9] = np.nan      # left wrist unseen for 8 frames
        p2[:6, :, 15] = np.nan                    # left ankle seen by 2 cameras only
    init = o.triangulate(p2.reshape(8, -1, 2)).reshape(F, 17, 3)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    return cams, o, p2, init, cons, weak, skel[0]


def _oracle_cost(o, x, p2, cons, weak, ssf, args, loss="soft_l1"):
    r = o._error_fun_triangulation(x, p2, np.array(cons), np.array(weak), ssf, args["scale_length"],
                                   args["scale_length_weak"], args["reproj_error_threshold"], loss,
                                   args["n_deriv_smooth"])
    return 0.5 * np.sum(r ** 2)


SOLVERS = ["trf", "lm"]


def _check_against_scipy(F, drop=0.1, gap=False, args=ARGS, loss="soft_l1", solver="trf"):
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch
    from oracle.geometry import optim_points
    cams, o, p2, init, cons, weak, truth = _problem(F, drop, gap)
    sa = optim_points(o, p2, init, cons, weak, reproj_loss=loss, ftol=1e-3, return_result=True, **args)
    sb = optim_points(o, p2, init, cons, weak, reproj_loss=loss, ftol=1e-10, return_result=True, **args)
    g = CameraGroup.from_dicts(cams)
    p3g, jlg, st, _ = optim_points_batch(g, p2[None], init[None], cons, weak, reproj_loss=loss, solver=solver,
                                         return_stats=True, **args)
    p3g, jlg = p3g[0], jlg[0]
    p3a, p3b = sa[0], sb[0]
    band = np.linalg.norm(p3a - p3b, axis=-1)
    dev = np.linalg.norm(p3g - p3a, axis=-1)
    assert np.median(dev) <= max(np.median(band), 1.0), (np.median(dev), np.median(band))
    assert np.percentile(dev, 99) <= max(np.percentile(band, 99), 5.0), (np.percentile(dev, 99),
                                                                          np.percentile(band, 99))
    if solver == "trf":  # scipy's own stopping point, not just a point of its band
        assert np.median(dev) <= 1.0 and np.percentile(dev, 99) <= 5.0, (np.median(dev), np.percentile(dev, 99))
        assert abs(st[0, 5] - sa[2].njev) <= 1, (st[0], sa[2].njev, sa[2].nfev)
    ssf = sa[3]
    xg = np.hstack([p3g.ravel(), jlg])
    cg = _oracle_cost(o, xg, p2, cons, weak, ssf, args, loss)
    assert cg <= sa[2].cost * (1 + 1e-3), (cg, sa[2].cost, sb[2].cost)
    np.testing.assert_allclose(jlg, sa[1], rtol=0.02, atol=1.0)
    return p3g, jlg


@pytest.mark.parametrize("solver", SOLVERS)
def test_optim_points_matches_scipy(solver):
    _check_against_scipy(40, solver=solver)


@pytest.mark.parametrize("solver", SOLVERS)
def test_optim_points_with_gaps_and_sparse_views(solver):
    _check_against_scipy(36, drop=0.3, gap=True, solver=solver)


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("loss,n", [("huber", 2), ("linear", 1)])
def test_optim_points_loss_and_order_variants(loss, n, solver):
    args = dict(ARGS, n_deriv_smooth=n)
    _check_against_scipy(24, args=args, loss=loss, solver=solver)


@pytest.mark.parametrize("F,n", [(2, 2), (3, 2), (4, 1), (5, 3)])
def test_optim_points_trf_short_clips(F, n):
    """Clips shorter than or barely longer than the smoothing order (no or one smoothness row per joint): the trf
    solver against scipy at the same bounds.  (One frame fails inside the reference's own setup -- numpy's mean
    of an empty difference -- so it is not a case.)"""
    args = dict(ARGS, n_deriv_smooth=n)
    _check_against_scipy(F, args=args, solver="trf")


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("F", [20, 100])
def test_optim_batch_equals_single_and_is_deterministic(solver, F):
    """An animal's result does not depend on the animals that share its call, bit for bit (the trf solver's
    frames per workgroup follow F, not the batch: at 100 frames a batch-sized grid would have picked 2 frames
    per workgroup for 3 animals and 1 for one)."""
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch
    probs = [_problem(F, seed=s) for s in (3, 4, 5)]
    cams = probs[0][0]
    g = CameraGroup.from_dicts(cams)
    P2 = np.stack([p[2] for p in probs])
    I3 = np.stack([p[3] for p in probs])
    cons, weak = probs[0][4], probs[0][5]
    a, la = optim_points_batch(g, P2, I3, cons, weak, solver=solver, **ARGS)
    b, lb = optim_points_batch(g, P2, I3, cons, weak, solver=solver, **ARGS)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(la, lb)
    for i in range(3):
        s, ls = optim_points_batch(g, P2[i:i + 1], I3[i:i + 1], cons, weak, solver=solver, **ARGS)
        np.testing.assert_array_equal(s[0], a[i])
        np.testing.assert_array_equal(ls[0], la[i])


def test_optim_points_jointlenfix_keeps_lengths_and_lowers_cost():
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch, prepare_batch
    cams, o, p2, init, cons, weak, truth = _problem(30)
    g = CameraGroup.from_dicts(cams)
    jl_fixed = np.linspace(60, 300, len(cons) + len(weak))
    p3, jl = g.optim_points_jointlenfix(p2, init, jl_fixed, constraints=cons, constraints_weak=weak, **ARGS)
    np.testing.assert_array_equal(jl, jl_fixed)
    x0, ssf = prepare_batch(init[None], cons, weak, ARGS["scale_smooth"])
    x0, ssf = x0[0], ssf[0]
    x0[-len(jl_fixed):] = jl_fixed
    c0 = _oracle_cost(o, x0, p2, cons, weak, ssf, ARGS)
    c1 = _oracle_cost(o, np.hstack([p3.ravel(), jl_fixed]), p2, cons, weak, ssf, ARGS)
    assert c1 < 0.5 * c0
    _, _, stats, _ = optim_points_batch(g, p2[None], init[None], cons, weak, joint_len=jl_fixed, max_iter=14,
                                        max_nfev=15, return_stats=True, **ARGS)
    assert stats[0, 4] <= 15 and stats[0, 2] <= 14
    _, _, stats, _ = optim_points_batch(g, p2[None], init[None], cons, weak, joint_len=jl_fixed, max_iter=14,
                                        solver="lm", return_stats=True, **ARGS)
    assert stats[0, 2] <= 14


@pytest.mark.parametrize("solver", SOLVERS)
@pytest.mark.parametrize("F,drop,gap", [(40, 0.1, False), (36, 0.3, True)])
def test_optim_points_jointlenfix_matches_scipy(F, drop, gap, solver):
    """optim_points_jointlenfix (cameras.py:1192-1415, max_nfev = 15) vs the oracle's scipy TRF run
    with the reference's arguments: same band / cost criteria as the free-length solve.  The fixed
    lengths are the clip's true median limb lengths (what calib/joint_len.npy holds in the reference)."""
    from mqhip.geometry import CameraGroup
    from oracle.geometry import optim_points_jointlenfix
    cams, o, p2, init, cons, weak, truth = _problem(F, drop, gap)
    jl = np.array([np.median(np.linalg.norm(truth[:, a] - truth[:, b], axis=1)) for a, b in cons + weak])
    sa = optim_points_jointlenfix(o, p2, init, jl, cons, weak, ftol=1e-3, max_nfev=15, return_result=True, **ARGS)
    sb = optim_points_jointlenfix(o, p2, init, jl, cons, weak, ftol=1e-10, max_nfev=None, return_result=True,
                                  **ARGS)
    g = CameraGroup.from_dicts(cams)
    from mqhip import optim as mqoptim
    prev = mqoptim.set_default_solver(solver)
    try:
        p3g, jlg = g.optim_points_jointlenfix(p2, init, jl, constraints=cons, constraints_weak=weak, **ARGS)
    finally:
        mqoptim.set_default_solver(prev)
    np.testing.assert_array_equal(jlg, jl)
    band = np.linalg.norm(sa[0] - sb[0], axis=-1)
    dev = np.linalg.norm(p3g - sa[0], axis=-1)
    assert np.median(dev) <= max(np.median(band), 1.0), (np.median(dev), np.median(band))
    assert np.percentile(dev, 99) <= max(np.percentile(band, 99), 5.0)
    cg = 0.5 * np.sum(o._error_fun_triangulation_jointlenfix(
        p3g.ravel(), p2, jl, np.array(cons), np.array(weak), sa[3], ARGS["scale_length"],
        ARGS["scale_length_weak"], ARGS["reproj_error_threshold"], "soft_l1", ARGS["n_deriv_smooth"]) ** 2)
    assert cg <= sa[2].cost * (1 + 1e-3), (cg, sa[2].cost, sb[2].cost)


@pytest.mark.parametrize("F,n", [(40, 2), (24, 1), (30, 3), (480, 2)])
def test_optim_precond_routes_agree(F, n):
    """(LM solver) The preconditioner has two kernels (optim.hip): the series staged in LDS with the two
    substitutions run by one lane quad (default when F (18 n + 9) doubles fit in 160 KB), and the
    global-memory kernel (MQ_TUNE_OPTIM_PRECOND_LDS = 0, and every clip longer than ~450 frames).  Both
    apply the same factor; rounding differs (fused products), so the solves agree to well inside the
    optim_points tolerance and the objectives to 1e-6 relative.  F = 480 runs the global kernel
    under both settings (bit-identical)."""
    from mqhip import _lib
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch
    cams, o, p2, init, cons, weak, truth = _problem(F)
    g = CameraGroup.from_dicts(cams)
    args = dict(ARGS, n_deriv_smooth=n)
    ctx = _lib.Context.get(0)
    old = ctx.lib.mq_get_tuning(18)
    try:
        out = {}
        for route in (1, 0):
            assert ctx.lib.mq_set_tuning(18, route) == 0
            out[route] = optim_points_batch(g, p2[None], init[None], cons, weak, return_stats=True, solver="lm",
                                            **args)
    finally:
        ctx.lib.mq_set_tuning(18, old)
    (a, la, sa, _), (b, lb, sb, _) = out[1], out[0]
    if F * (18 * n + 9) * 8 > 160 * 1024:
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(la, lb)
        return
    assert abs(sa[0, 1] - sb[0, 1]) <= 1e-6 * sb[0, 1], (sa[0], sb[0])
    dev = np.linalg.norm(a - b, axis=-1)
    assert np.nanmax(dev) < 0.05, np.nanmax(dev)
