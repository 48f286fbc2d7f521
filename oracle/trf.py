"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

CPU restatement of the solver the reference's optim_points runs: scipy.optimize.least_squares(method='trf',
jac_sparsity=..., loss='linear', ftol=1e-3) (/root/reference/src/third_party/aniposelib/cameras.py:1166-1180).
With no bounds and a sparse Jacobian that is scipy 1.15.3's ``trf_no_bounds`` with ``tr_solver='lsmr'``
(optimize/_lsq/trf.py:401-540): a damped lsmr Gauss-Newton step (the damping from the 1-D quadratic along -g,
``regularize=True``), the 2-D subspace {g, gn} orthonormalised by QR, ``solve_trust_region_2d``,
``update_tr_radius`` and ``check_termination``.  lsmr is sparse/linalg/_isolve/lsmr.py (atol = btol = 1e-6,
conlim 1e8, maxiter min(m, n)).

The restatement is written in the phase order of libmq_hip's TRF kernels (csrc/optim_trf.hip), so that the
device decomposition can be checked on the CPU:

  * lsmr keeps the raw vectors u_raw = A v - alpha u and v_raw = A^T u - beta v; each phase normalises its
    inputs by the previous phase's norm (scipy normalises in place: the same products);
  * the recurrences of iteration k run in the first phase of iteration k + 1 (that is where alpha_k is known),
    together with the x / h / hbar updates, and the stop test of iteration k runs in the second phase of
    iteration k + 1 (where ||x_k|| is known).  Moving a test later changes no value: x_k is final when
    iteration k's test passes, and the phases after it are not run.

With the same Jacobian and numpy's norms this reproduces scipy's ``least_squares`` bit for bit
(tests/test_oracle_trf.py pins it against scipy on the marker-scene problems).
"""
from __future__ import annotations

from math import sqrt

import numpy as np
from numpy.linalg import norm

EPS = np.finfo(float).eps


def sym_ortho(a, b):
    """scipy.sparse.linalg._isolve.lsqr._sym_ortho (lsqr.py:62-95)."""
    if b == 0:
        return np.sign(a), 0, abs(a)
    elif a == 0:
        return 0, np.sign(b), abs(b)
    elif abs(b) > abs(a):
        tau = a / b
        s = np.sign(b) / sqrt(1 + tau * tau)
        c = s * tau
        r = b / s
    else:
        tau = b / a
        c = np.sign(a) / sqrt(1 + tau * tau)
        s = c * tau
        r = a / c
    return c, s, r


def lsmr_phased(matvec, rmatvec, b, n, damp=0.0, atol=1e-6, btol=1e-6, conlim=1e8, maxiter=None):
    """lsmr (lsmr.py:29-460) in the kernels' phase order.  Returns (x, istop, itn)."""
    m = b.shape[0]
    if maxiter is None:
        maxiter = min(m, n)
    u = b
    normb = norm(b)
    x = np.zeros(n)
    beta = normb.copy()
    if beta > 0:
        u = (1 / beta) * u
        v = rmatvec(u)
        alpha = norm(v)
    else:
        v = np.zeros(n)
        alpha = 0
    if alpha > 0:
        v = (1 / alpha) * v
    # state (lsmr.py:205-239)
    zetabar = alpha * beta
    alphabar = alpha
    rho = rhobar = cbar = 1
    sbar = 0
    h = v.copy()
    hbar = np.zeros(n)
    betadd, betad, rhodold, tautildeold, thetatilde, zeta, d = beta, 0, 1, 0, 0, 0, 0
    normA2 = alpha * alpha
    maxrbar, minrbar = 0, 1e+100
    ctol = 1 / conlim if conlim > 0 else 0
    if alpha * beta == 0 or normb == 0:
        return x, 0, 0
    itn = 0
    pending = None      # iteration k's scalars, tested in phase 2 of iteration k + 1
    while True:
        # ---- phase 1 of iteration itn + 1: u = A v - alpha u (v, u normalised by the previous phase's norms)
        if itn >= maxiter:
            break
        itn += 1
        u = u * -alpha
        u = u + matvec(v)
        beta = norm(u)
        # ---- phase 2: the test of the previous iteration (its x is final if it passes), then v = A^T u - beta v
        if pending is not None and pending[0]:
            itn -= 1
            return x, pending[1], itn
        if beta > 0:
            u = u * (1 / beta)
            v = v * -beta
            v = v + rmatvec(u)
            alpha = norm(v)
            if alpha > 0:
                v = v * (1 / alpha)
        # ---- phase 1 of the next iteration: this iteration's recurrences and the x / h / hbar updates
        chat, shat, alphahat = sym_ortho(alphabar, damp)
        rhoold = rho
        c, s, rho = sym_ortho(alphahat, beta)
        thetanew = s * alpha
        alphabar = c * alpha
        rhobarold = rhobar
        zetaold = zeta
        thetabar = sbar * rho
        rhotemp = cbar * rho
        cbar, sbar, rhobar = sym_ortho(cbar * rho, thetanew)
        zeta = cbar * zetabar
        zetabar = - sbar * zetabar
        hbar = hbar * -(thetabar * rho / (rhoold * rhobarold))
        hbar = hbar + h
        x = x + (zeta / (rho * rhobar)) * hbar
        h = h * -(thetanew / rho)
        h = h + v
        betaacute = chat * betadd
        betacheck = -shat * betadd
        betahat = c * betaacute
        betadd = -s * betaacute
        thetatildeold = thetatilde
        ctildeold, stildeold, rhotildeold = sym_ortho(rhodold, thetabar)
        thetatilde = stildeold * rhobar
        rhodold = ctildeold * rhobar
        betad = - stildeold * betad + ctildeold * betahat
        tautildeold = (zetaold - thetatildeold * tautildeold) / rhotildeold
        taud = (zeta - thetatilde * tautildeold) / rhodold
        d = d + betacheck * betacheck
        normr = sqrt(d + (betad - taud) ** 2 + betadd * betadd)
        normA2 = normA2 + beta * beta
        normA = sqrt(normA2)
        normA2 = normA2 + alpha * alpha
        maxrbar = max(maxrbar, rhobarold)
        if itn > 1:
            minrbar = min(minrbar, rhobarold)
        condA = max(maxrbar, rhotemp) / min(minrbar, rhotemp)
        normar = abs(zetabar)
        normx = norm(x)            # phase 2 of the next iteration reduces ||x||
        test1 = normr / normb
        test2 = normar / (normA * normr) if (normA * normr) != 0 else np.inf
        test3 = 1 / condA
        t1 = test1 / (1 + normA * normx / normb)
        rtol = btol + atol * normA * normx / normb
        istop = 0
        if itn >= maxiter:
            istop = 7
        if 1 + test3 <= 1:
            istop = 6
        if 1 + test2 <= 1:
            istop = 5
        if 1 + t1 <= 1:
            istop = 4
        if test3 <= ctol:
            istop = 3
        if test2 <= atol:
            istop = 2
        if test1 <= rtol:
            istop = 1
        pending = (istop > 0, istop)
        if istop > 0 and itn >= maxiter:
            return x, istop, itn
    return x, 7, itn


def solve_trust_region_2d(B, g, Delta):
    """optimize/_lsq/common.py solve_trust_region_2d: the Newton step if it lies inside, else the boundary
    minimum from the quartic in t = tan(phi / 2) (numpy.roots)."""
    from numpy.linalg import LinAlgError
    from scipy.linalg import cho_factor, cho_solve
    try:
        R, lower = cho_factor(B)
        p = -cho_solve((R, lower), g)
        if np.dot(p, p) <= Delta ** 2:
            return p, True
    except LinAlgError:
        pass
    a = B[0, 0] * Delta ** 2
    b = B[0, 1] * Delta ** 2
    c = B[1, 1] * Delta ** 2
    d = g[0] * Delta
    f = g[1] * Delta
    coeffs = np.array([-b + d, 2 * (a - c + f), 6 * b, 2 * (-a + c + f), -b - d])
    t = np.roots(coeffs)
    t = np.real(t[np.isreal(t)])
    p = Delta * np.vstack((2 * t / (1 + t ** 2), (1 - t ** 2) / (1 + t ** 2)))
    value = 0.5 * np.sum(p * B.dot(p), axis=0) + np.dot(g, p)
    i = np.argmin(value)
    return p[:, i], False


def update_tr_radius(Delta, actual_reduction, predicted_reduction, step_norm, bound_hit):
    """common.py update_tr_radius."""
    if predicted_reduction > 0:
        ratio = actual_reduction / predicted_reduction
    elif predicted_reduction == actual_reduction == 0:
        ratio = 1
    else:
        ratio = 0
    if ratio < 0.25:
        Delta = 0.25 * step_norm
    elif ratio > 0.75 and bound_hit:
        Delta *= 2.0
    return Delta, ratio


def check_termination(dF, F, dx_norm, x_norm, ratio, ftol, xtol):
    """common.py check_termination."""
    ftol_satisfied = dF < ftol * F and ratio > 0.25
    xtol_satisfied = dx_norm < xtol * (xtol + x_norm)
    if ftol_satisfied and xtol_satisfied:
        return 4
    elif ftol_satisfied:
        return 2
    elif xtol_satisfied:
        return 3
    return None


def trf_no_bounds(fun, jac, x0, ftol=1e-3, xtol=1e-8, gtol=1e-8, max_nfev=None, lsmr_log=None):
    """trf.py:401-540 with x_scale = 1, loss 'linear', tr_solver 'lsmr', regularize True, damp 0.
    ``jac(x, f)`` returns a scipy sparse matrix (or anything with .dot / .T.dot).
    Returns (x, cost, nfev, njev, status)."""
    from scipy.linalg import qr
    x = x0.copy()
    f = fun(x)
    nfev = 1
    J = jac(x, f)
    njev = 1
    m, n = J.shape
    cost = 0.5 * np.dot(f, f)
    g = J.T.dot(f)
    Delta = norm(x0)
    if Delta == 0:
        Delta = 1.0
    if max_nfev is None:
        max_nfev = x0.size * 100
    termination_status = None
    while True:
        g_norm = norm(g, ord=np.inf)
        if g_norm < gtol:
            termination_status = 1
        if termination_status is not None or nfev == max_nfev:
            break
        g_h = g
        # regularize: the 1-D quadratic along -g inside the trust region
        v = J.dot(-g_h)
        a = 0.5 * np.dot(v, v)
        b = np.dot(g_h, -g_h)
        to_tr = Delta / norm(g_h)
        ts = [0, to_tr]
        if a != 0:
            ext = -0.5 * b / a
            if 0 < ext < to_tr:
                ts.append(ext)
        ts = np.asarray(ts)
        ag_value = np.min(ts * (a * ts + b))
        reg_term = -ag_value / Delta ** 2
        damp_full = (0.0 ** 2 + reg_term) ** 0.5
        gn_h, istop, itn = lsmr_phased(lambda z: J.dot(z), lambda z: J.T.dot(z), f, n, damp=damp_full)
        if lsmr_log is not None:
            lsmr_log.append(itn)
        S = np.vstack((g_h, gn_h)).T
        S, _ = qr(S, mode='economic')
        JS = J.dot(S)
        B_S = np.dot(JS.T, JS)
        g_S = S.T.dot(g_h)
        actual_reduction = -1
        while actual_reduction <= 0 and nfev < max_nfev:
            p_S, _ = solve_trust_region_2d(B_S, g_S, Delta)
            step_h = S.dot(p_S)
            Js = J.dot(step_h)
            predicted_reduction = -(0.5 * np.dot(Js, Js) + np.dot(step_h, g_h))
            step = step_h
            x_new = x + step
            f_new = fun(x_new)
            nfev += 1
            step_h_norm = norm(step_h)
            if not np.all(np.isfinite(f_new)):
                Delta = 0.25 * step_h_norm
                continue
            cost_new = 0.5 * np.dot(f_new, f_new)
            actual_reduction = cost - cost_new
            Delta_new, ratio = update_tr_radius(Delta, actual_reduction, predicted_reduction, step_h_norm,
                                                step_h_norm > 0.95 * Delta)
            step_norm = norm(step)
            termination_status = check_termination(actual_reduction, cost, step_norm, norm(x), ratio, ftol, xtol)
            if termination_status is not None:
                break
            Delta = Delta_new
        if actual_reduction > 0:
            x = x_new
            f = f_new
            cost = cost_new
            J = jac(x, f)
            njev += 1
            g = J.T.dot(f)
    if termination_status is None:
        termination_status = 0
    return x, cost, nfev, njev, termination_status
