"""CPU: host-side pieces of the drop-in mirror against the oracle (no GPU needed)."""
import numpy as np


def test_optim_prepare_matches_oracle_init():
    """x0 and scale_smooth_full (cameras.py:1125-1150) are bit-identical to the oracle's."""
    from mqhip import synth
    from mqhip.optim import prepare
    from oracle.geometry import initialize_params_triangulation, interpolate_data, medfilt_data
    rng = np.random.default_rng(0)
    p3 = synth.make_skeletons(1, 50)[0] + rng.normal(0, 3, (50, 17, 3))
    p3[rng.random((50, 17)) < 0.2] = np.nan
    p3[:, 4] = np.nan                                 # a joint never triangulated
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    x0, ssf = prepare(p3, cons, weak, 3)
    intp = np.apply_along_axis(interpolate_data, 0, p3)
    med = np.apply_along_axis(medfilt_data, 0, intp, size=7)
    ref_ssf = 3 * (1.0 / np.mean(np.abs(np.diff(med, axis=0))))
    ref_x0 = initialize_params_triangulation(intp, np.array(cons), np.array(weak))
    ref_x0[~np.isfinite(ref_x0)] = 0
    np.testing.assert_array_equal(x0, ref_x0)
    assert ssf == ref_ssf
