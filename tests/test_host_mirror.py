"""CPU: host-side pieces of the drop-in mirror against the oracle (no GPU needed)."""
import numpy as np
import pytest


@pytest.mark.parametrize("F,ties", [(50, False), (300, False), (300, True)])
def test_optim_prepare_matches_oracle_init(F, ties):
    """x0 and scale_smooth_full (cameras.py:1125-1150) from libmq_hip's host initialisation
    (mq_optim_prepare through mqhip.optim.prepare_batch) are bit-identical to the oracle's; ties
    exercise the order-statistic median."""
    from mqhip import synth
    from mqhip.optim import prepare_batch
    from oracle.geometry import initialize_params_triangulation, interpolate_data, medfilt_data
    rng = np.random.default_rng(F)
    p3 = synth.make_skeletons(1, F)[0] + rng.normal(0, 3, (F, 17, 3))
    if ties:
        p3 = np.round(p3 / 4) * 4
    p3[rng.random((F, 17)) < 0.2] = np.nan
    p3[:, 4] = np.nan                                 # a joint never triangulated
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    x0, ssf = prepare_batch(p3[None], cons, weak, 3)
    x0, ssf = x0[0], ssf[0]
    intp = np.apply_along_axis(interpolate_data, 0, p3)
    med = np.apply_along_axis(medfilt_data, 0, intp, size=7)
    ref_ssf = 3 * (1.0 / np.mean(np.abs(np.diff(med, axis=0))))
    ref_x0 = initialize_params_triangulation(intp, np.array(cons), np.array(weak))
    ref_x0[~np.isfinite(ref_x0)] = 0
    np.testing.assert_array_equal(x0, ref_x0)
    assert ssf == ref_ssf


def _rng_boxes(rng, n):
    x1 = rng.integers(0, 1800, n)
    y1 = rng.integers(0, 1300, n)
    w = rng.integers(-3, 400, n)
    h = rng.integers(-3, 400, n)
    tr = np.stack([x1 + rng.random(n), y1 + rng.random(n), x1 + w + rng.random(n), y1 + h + rng.random(n),
                   rng.integers(1, 9, n), rng.random(n)], axis=1)
    return tr


def test_step1_box_filter_and_expansion_match_oracle():
    """Rows a1 + the degenerate-box filter (step1:255-292), bit-exact vs the per-box oracle."""
    from oracle import postprocess as op
    from src.pipeline import step1_proc2d as s1
    rng = np.random.default_rng(1)
    tr = _rng_boxes(rng, 400)
    b, t = s1.filter_tracks(tr)
    ob, ot = op.filter_tracks(tr)
    np.testing.assert_array_equal(b, ob)
    np.testing.assert_array_equal(t, ot)
    np.testing.assert_array_equal(s1.expand_boxes(b), op.expand_boxes(ob))
    assert s1.filter_tracks(np.zeros((0, 7)))[0].shape == (0, 4)


def test_step1_keypoint_threshold_and_ema_match_oracle():
    """Row a10: KP_THR masking + recursive EMA over per-track deques, bit-exact vs the oracle."""
    from types import SimpleNamespace
    from oracle import postprocess as op
    from src.pipeline import step1_proc2d as s1
    rng = np.random.default_rng(2)
    sm, osm = s1.KeypointSmoother(), op.Smoother()
    base = rng.uniform(100, 1500, (3, 17, 2))
    for fn in range(40):
        tids = rng.permutation([3, 5, 9])[:rng.integers(1, 4)]
        kps = np.stack([base[[3, 5, 9].index(t)] + rng.normal(0, 12, (17, 2)) for t in tids])
        sc = rng.uniform(0, 1, (len(tids), 17)).astype(np.float32)
        boxes = np.tile(np.array([[10, 20, 200, 300]], np.int32), (len(tids), 1))
        res = [SimpleNamespace(pred_instances=SimpleNamespace(keypoints=kps[i][None], keypoint_scores=sc[i][None]))
               for i in range(len(tids))]
        rows = s1._rows(res, boxes, tids, sm, fn, None, s1.KP_PARAMS)
        orows = op.frame_rows(kps, sc, boxes, tids, osm, fn)
        assert len(rows) == len(orows)
        for r, o in zip(rows, orows):
            assert r[:5] == o[:5] and r[6:] == o[6:]
            np.testing.assert_array_equal(np.array(r[5]), np.array(o[5]))
