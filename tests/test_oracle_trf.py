"""CPU: oracle/trf.py (scipy's trf_no_bounds + lsmr restated in the phase order of csrc/optim_trf.hip) against
scipy.optimize.least_squares itself, and the optim_points fixture against scipy run here.

* With scipy's own 2-point sparse Jacobian, the restatement reproduces least_squares bit for bit (x, nfev,
  njev): the phase reordering of lsmr (raw vectors normalised by the next phase, the recurrences of iteration k
  run in phase 1 of k + 1, the stop test of k in phase 2 of k + 1) changes no value.
* tests/golden/optim_problems.npz (dumped on the GPU box by tools/dump_optim_problems.py) holds scipy's answers:
  re-running scipy here gives the same bits.
"""
import os

import numpy as np
import pytest

FIX = os.path.join(os.path.dirname(__file__), "golden", "optim_problems.npz")


def _problem(key):
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle, jac_sparsity_triangulation, optim_init
    z = np.load(FIX)
    ss, sl, slw, rp, nd = z["tri"]
    o = CameraGroupOracle(synth.make_cameras(8))
    p2, init = z[key + "_p2"], z[key + "_init"]
    x0, ssf = optim_init(init, z["cons"], z["weak"], ss)
    sp = jac_sparsity_triangulation(p2, z["cons"], z["weak"], int(nd))
    args = (p2, z["cons"], z["weak"], ssf, sl, slw, rp, "soft_l1", int(nd))
    return z, o, x0, sp, args


@pytest.mark.parametrize("key", ["s7f8a1", "s7f8a3"])
def test_trf_restatement_is_scipy_bit_for_bit(key):
    from scipy import optimize
    from scipy.optimize._numdiff import approx_derivative, group_columns
    from oracle import trf as otrf
    z, o, x0, sp, args = _problem(key)
    fun = lambda x: o._error_fun_triangulation(x, *args)  # noqa: E731
    spg = (sp, group_columns(sp))
    jac = lambda x, f: approx_derivative(fun, x, method="2-point", f0=f, bounds=(-np.inf, np.inf),  # noqa: E731
                                         sparsity=spg)
    x, cost, nfev, njev, status = otrf.trf_no_bounds(fun, jac, x0, ftol=1e-3)
    ref = optimize.least_squares(o._error_fun_triangulation, x0=x0, jac_sparsity=sp, loss="linear", ftol=1e-3,
                                 args=args)
    np.testing.assert_array_equal(x, ref.x)
    assert (nfev, njev, status) == (ref.nfev, ref.njev, ref.status)
    assert cost == ref.cost


@pytest.mark.parametrize("key", ["s7f8a0", "s7f8a2"])
def test_fixture_holds_scipys_answer(key):
    from scipy import optimize
    z, o, x0, sp, args = _problem(key)
    ref = optimize.least_squares(o._error_fun_triangulation, x0=x0, jac_sparsity=sp, loss="linear", ftol=1e-3,
                                 args=args)
    np.testing.assert_array_equal(ref.x, z[key + "_x"])
    assert (ref.nfev, ref.njev) == tuple(int(v) for v in z[key + "_stats"][:2])


def test_solve_trust_region_2d_and_lsmr_pieces():
    """Known answers of the 2-D subproblem (inside -> Newton step; outside -> on the boundary, the minimum of
    the quadratic over the circle, checked against a dense angle scan) and of lsmr on a small dense system."""
    from oracle import trf as otrf
    B = np.array([[4.0, 1.0], [1.0, 3.0]])
    g = np.array([1.0, 2.0])
    p, newton = otrf.solve_trust_region_2d(B, g, 10.0)
    assert newton
    np.testing.assert_allclose(p, -np.linalg.solve(B, g), rtol=1e-14)
    p, newton = otrf.solve_trust_region_2d(B, g, 0.1)
    assert not newton and abs(np.linalg.norm(p) - 0.1) < 1e-12
    ang = np.linspace(0, 2 * np.pi, 200001)
    q = 0.1 * np.stack([np.cos(ang), np.sin(ang)])
    vals = 0.5 * np.sum(q * (B @ q), axis=0) + g @ q
    assert 0.5 * p @ B @ p + g @ p <= vals.min() + 1e-9
    rng = np.random.default_rng(0)
    A = rng.standard_normal((40, 12))
    b = rng.standard_normal(40)
    x, istop, itn = otrf.lsmr_phased(A.dot, A.T.dot, b, 12, atol=1e-12, btol=1e-12)
    np.testing.assert_allclose(x, np.linalg.lstsq(A, b, rcond=None)[0], rtol=1e-8, atol=1e-10)
    from scipy.sparse.linalg import lsmr
    ref = lsmr(A, b, damp=0.3)
    x, istop, itn = otrf.lsmr_phased(A.dot, A.T.dot, b, 12, damp=0.3)
    np.testing.assert_array_equal(x, ref[0])
    assert (istop, itn) == (ref[1], ref[2])
