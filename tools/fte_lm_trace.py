"""Iterate-by-iterate comparison of the GPU FTE solve with the oracle LM on a start that
forces rejected steps: python tools/fte_lm_trace.py [const|variable] [iters] [angle_offset].
For k = 1..iters it runs acs_fte_solve with max_iters = k and prints the oracle's and the
GPU's accept count, cost and the max |X_gpu - X_oracle| after k iterations."""
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from oracle import fte as ofte  # noqa: E402
from acinoset_amd import _native, kinematics as pkin  # noqa: E402
from test_gpu_fte import _problem  # noqa: E402


def oracle_history(prob, X0, iters, lam0=1e-3, tau0=None):
    X = np.array(X0, np.float64)
    tau = np.zeros(prob.tau_shape) if tau0 is None else np.array(tau0, np.float64)
    F, H, g = prob.linearize(X, tau)
    lam, nacc, hist = lam0, 0, []
    pin0 = prob.pinned() if prob.sd else None
    for it in range(iters):
        pin, gp = None, g
        if pin0 is not None:
            pin = np.concatenate([pin0, ofte.active_bounds(prob, tau, g)])
            gp = g.copy()
            gp[pin] = 0.0
        A = (H + sp.diags(lam * np.maximum(H.diagonal(), 1e-12))).tolil()
        if pin is not None:
            A[pin, :] = 0.0
            A[:, pin] = 0.0
            A[pin, pin] = 1.0
        d = spla.spsolve(A.tocsc(), -gp)
        dX, dtau = prob.unpack(d)
        Xn = X + dX
        taun = np.clip(tau + dtau, -prob.Ts, prob.Ts) if prob.sd else tau
        if prob.sd:
            taun[..., 0] = 0.0
        Fn = prob.cost(Xn, taun)[0]
        acc = Fn < F
        if acc:
            nacc += 1
            X, tau = Xn, taun
            lam = max(lam * 0.1, 1e-15)
            F, H, g = prob.linearize(X, tau)
        else:
            lam *= 10.0
        hist.append((X.copy(), tau.copy(), F, Fn, lam, nacc, acc))
    return hist


if __name__ == '__main__':
    mode = sys.argv[1] if len(sys.argv) > 1 else 'const'
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    off = float(sys.argv[3]) if len(sys.argv) > 3 else 1.5
    N = 40
    seq, prob, cams = _problem(N, sd_mode=mode)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0]).copy()
    X0[:, 3:] += off
    hist = oracle_history(prob, X0, iters)
    ctx = _native.Context(0)
    table = pkin.build_table(prob.mode)
    restart = int(os.environ.get('RESTART', '0'))
    if restart:
        # both sides restarted from the oracle's iterate `restart` with its lambda: isolates
        # solver differences from the growth of rounding differences along the path
        Xr, tr, Fr, _, lamr, _, _ = hist[restart - 1]
        hr = oracle_history(prob, Xr, 8, lam0=lamr, tau0=tr)
        for k in range(1, 9):
            o = ctx.fte_default_opts(max_iters=k, ftol=0.0, xtol=0.0, gtol=0.0, lambda0=lamr)
            X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, Xr, tau0=tr, opts=o,
                                        sd_mode=mode)
            Xo, to, Fo, Fno, lamo, nacco, acco = hr[k - 1]
            print(f'restart {restart} k {k} oracle acc={int(acco)} F {Fo:.12e} trialF {Fno:.8e} | gpu nacc '
                  f'{rep["n_accepted"]} F {rep["cost_after"]:.12e} | max|dX| {np.abs(X - Xo).max():.2e}', flush=True)
        # one step at the lambda of restart step 5, fresh (no preceding rejections): the
        # GPU step's backward error in the oracle's damped system
        lam5 = hr[3][4]
        o = ctx.fte_default_opts(max_iters=1, ftol=0.0, xtol=0.0, gtol=0.0, lambda0=lam5)
        X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, Xr, tau0=tr, opts=o,
                                    sd_mode=mode)
        F, H, g = prob.linearize(Xr, tr)
        pin = np.concatenate([prob.pinned(), ofte.active_bounds(prob, tr, g)])
        g = g.copy()
        g[pin] = 0.0
        A = (H + sp.diags(lam5 * np.maximum(H.diagonal(), 1e-12))).tolil()
        A[pin, :] = 0.0
        A[:, pin] = 0.0
        A[pin, pin] = 1.0
        A = A.tocsc()
        d_or = spla.spsolve(A, -g)
        d_gpu = prob.pack(X, tau) - prob.pack(Xr, tr)
        for name, d in (('oracle', d_or), ('gpu', d_gpu)):
            r = A @ d + g
            print(f'lam {lam5:.0e} {name}: |A d + g| / |g| = {np.linalg.norm(r) / np.linalg.norm(g):.3e}  '
                  f'|d| = {np.linalg.norm(d):.4e}  cost {prob.cost(*prob.unpack(d + prob.pack(Xr, tr)))[0]:.8e}',
                  flush=True)
        print(f'gpu fresh one step at lam {lam5:.0e}: nacc {rep["n_accepted"]} F {rep["cost_after"]:.10e}; '
              f'|d_gpu - d_or| = {np.linalg.norm(d_gpu - d_or):.3e}')
        ev = np.linalg.eigvalsh(A.toarray())
        print(f'damped matrix eigenvalues: min {ev[0]:.3e} max {ev[-1]:.3e} cond {ev[-1] / ev[0]:.3e}')
        sys.exit(0)
    for k in range(1, iters + 1):
        X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                    opts=ctx.fte_default_opts(max_iters=k, ftol=0.0, xtol=0.0, gtol=0.0),
                                    sd_mode=mode)
        Xo, to, Fo, Fno, lamo, nacco, acco = hist[k - 1]
        print(f'k {k:3d} oracle acc={int(acco)} nacc {nacco:3d} F {Fo:.12e} trialF {Fno:.6e} lam {lamo:.0e} | '
              f'gpu nacc {rep["n_accepted"]:3d} F {rep["cost_after"]:.12e} lam {rep["lambda_final"]:.0e} | '
              f'max|dX| {np.abs(X - Xo).max():.2e} max|dtau| {np.abs(tau - to).max():.2e}', flush=True)
