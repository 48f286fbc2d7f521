"""GPU: the end-to-end tolerance north_star asks for -- 3D joints of the HIP chain against the oracle chain
from identical frames and weights (tests/parity3d.py has the two chains and the definitions).

Cases: BASELINE config 2 (one frame, 8 views x 4 individuals, ViTPose-H, DLT: optim_points needs >= 20
points per individual, step4:242-245) and a 24-frame slice of the config-4 clip through the reference's
default step 4 (Viterbi -> DLT -> optim_points, ``ransac = false``).  Stated tolerances:
  * argmax bit-exact on every clear joint (top-2 margin > 5e-2 max|H|);
  * the clear fraction is at least CLEAR_MIN (random-weight heatmaps have flat tops; the figure is the
    share of joints the bit-exact statement covers);
  * keypoints within 0.5 px on clear, Taylor-regime joints;
  * on all-clear points (every kept view clear, both chains keep the same views; at least ALL_CLEAR_MIN):
    the DLT of the score-thresholded views within KP3D_DLT_MM_MEDIAN / KP3D_DLT_MM_P99 mm (median / p99) --
    the bf16 path's 2D differences carried into 3D; and, where optim_points ran (the reference default,
    >= 20 points per individual), GPU LM and scipy TRF stop early at different points of the same problem,
    so: the GPU solver on the oracle chain's own 2D costs at most SOLVER_COST_RATIO x scipy's; the HIP
    chain's solution, scored by the oracle's objective on the oracle's inputs, at most OPTIM_COST_RATIO x;
    both lie within max(scipy's own ftol 1e-3 vs 1e-10 band, KP3D_OPTIM_MM_MEDIAN / KP3D_OPTIM_MM_P99) of
    the converged (ftol 1e-10) solution; the chains' optimised joints differ by at most
    KP3D_OPTIM_E2E_MM_MEDIAN mm (median).
"""
import json

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def weights():
    import parity3d
    return parity3d.make_weights()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_frames,seed", [(1, 7), (24, 7), (24, 8), (24, 9)])
def test_parity_3d_hip_chain_vs_oracle_chain(weights, n_frames, seed):
    """Seeds 8 and 9 are further marker scenes (other skeletons and marker noise) for the same statements:
    the ABI-5 solver stop missed SOLVER_COST_RATIO on seed 8 (1.015x), the ABI-6 one passes all three
    (profiles/r04p_parity3d_seeds_8_9.log, r04t_parity3d_seeds_8_9_abi6.log)."""
    import parity3d
    fig, hip, ora = parity3d.run(n_frames=n_frames, seed=seed, weights=weights)
    print("parity3d", json.dumps(fig))
    assert fig["argmax_equal_on_clear"] == 1.0
    assert fig["clear_fraction"] >= parity3d.CLEAR_MIN
    assert fig["n_clear_taylor_scored"] > 0 and fig["kp_max_abs_px"] <= parity3d.KP_TOL_PX
    assert fig["all_clear_points"] >= parity3d.ALL_CLEAR_MIN
    assert fig["kp3d_dlt_mm_all_clear_median"] <= parity3d.KP3D_DLT_MM_MEDIAN
    assert fig["kp3d_dlt_mm_all_clear_p99"] <= parity3d.KP3D_DLT_MM_P99
    if fig["optim_points"]:
        # the GPU optim_points against scipy on the oracle chain's own (ViT-derived) 2D inputs: cost within
        # 0.1 % of scipy's, and no farther from the converged solution than scipy's own ftol-1e-3 stop is
        assert fig["solver_cost_ratio_max"] <= parity3d.SOLVER_COST_RATIO
        assert fig["solver_to_converged_mm_median"] <= max(fig["scipy_band_all_mm_median"], parity3d.KP3D_OPTIM_MM_MEDIAN)
        assert fig["solver_to_converged_mm_p99"] <= max(fig["scipy_band_all_mm_p99"], parity3d.KP3D_OPTIM_MM_P99)
        # end to end (each chain its own 2D): the same two statements on all-clear points, and the median
        # distance between the chains' optimised joints
        assert fig["optim_cost_ratio_max"] <= parity3d.OPTIM_COST_RATIO
        assert fig["kp3d_optim_to_converged_mm_median"] <= max(fig["scipy_band_mm_median"], parity3d.KP3D_OPTIM_MM_MEDIAN)
        assert fig["kp3d_optim_to_converged_mm_p99"] <= max(fig["scipy_band_mm_p99"], parity3d.KP3D_OPTIM_MM_P99)
        assert fig["kp3d_optim_mm_all_clear_median"] <= parity3d.KP3D_OPTIM_E2E_MM_MEDIAN
