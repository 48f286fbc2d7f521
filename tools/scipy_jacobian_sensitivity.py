"""How far scipy's own optim_points answer moves when its 2-point finite-difference Jacobian is replaced by
3-point differences (a near-analytic Jacobian), per marker-scene problem of tests/golden/optim_problems.npz: the
floor of what any restatement with an analytic Jacobian can be held to.  Also logs lsmr's iterations per call.
python tools/scipy_jacobian_sensitivity.py [problem keys]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"), os.path.join(ROOT, "tests")]
from mqhip import synth
from oracle import geometry as og
from scipy import optimize
import scipy.optimize._lsq.trf as trf
from scipy.sparse.linalg import lsmr as _lsmr
Z = np.load(os.path.join(ROOT, "tests", "golden", "optim_problems.npz"))
cons, weak = Z["cons"], Z["weak"]; ss, sl, slw, rp, nd = Z["tri"]; nd = int(nd)
LOG = []
def lsmr_log(*a, **k):
    r = _lsmr(*a, **k); LOG.append(r[2]); return r
trf.lsmr = lsmr_log
keys = sorted({k.rsplit("_", 1)[0] for k in Z.files if k.startswith("s")})
sel = sys.argv[1:] or keys
cache = {}
for key in sel:
    seed = int(key[1:key.index("f")])
    if seed not in cache: cache[seed] = og.CameraGroupOracle(synth.make_cameras(8))
    o = cache[seed]
    p2, init = Z[key + "_p2"], Z[key + "_init"]
    F = p2.shape[1]; J = p2.shape[2]
    x0, ssf = og.optim_init(init, cons, weak, ss)
    sp = og.jac_sparsity_triangulation(p2, cons, weak, nd)
    out = {}
    for jac in ("2-point", "3-point"):
        LOG.clear()
        r = optimize.least_squares(o._error_fun_triangulation, x0=x0, jac_sparsity=sp, jac=jac, loss='linear', ftol=1e-3,
            args=(p2, cons, weak, ssf, sl, slw, rp, 'soft_l1', nd))
        out[jac] = (r, list(LOG))
    r2, r3 = out["2-point"][0], out["3-point"][0]
    assert np.array_equal(r2.x, Z[key + "_x"]), "dump differs from the local scipy run"
    d = np.linalg.norm((r2.x - r3.x)[:F*J*3].reshape(-1, 3), axis=1)
    dt = np.linalg.norm(r2.x[:F*J*3].reshape(-1, 3) - Z[key + "_tight"].reshape(-1, 3), axis=1)
    print(key, "2pt nfev/njev", r2.nfev, r2.njev, "lsmr", out["2-point"][1], "| 3pt", r3.nfev, r3.njev, "lsmr", out["3-point"][1],
          "| d mm med/p99/max %.3f %.3f %.3f" % (np.median(d), np.percentile(d, 99), d.max()),
          "| cost ratio %.5f" % (r3.cost / r2.cost), "| band p99 %.2f" % np.nanpercentile(dt, 99), flush=True)
