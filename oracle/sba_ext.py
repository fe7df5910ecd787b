"""Oracle: sparse bundle adjustment of points AND camera extrinsics.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference: `bundle_adjust_points_and_extrinsics` (`src/lib/sba.py:158-178`): scipy
`least_squares(method='trf', loss='cauchy', f_scale=1 (default), ftol=1e-10,
max_nfev=1000, x_scale='jac')` over `cost_func_points_extrinsics` (:142-146) with
x = [Rodrigues vectors (C x 3), t (C x 3), points (n x 3)] and no gauge fix. In the survey
the reference stopped on xtol with first-order optimality 6.3e4 (not converged), so parity
is on the objective: the same robust cost, reached lower.

Same safeguarded LM as the GPU (acinoset_amd/csrc/sba_ext.hip):
  residual r = project(R_c X_i + t_c) - uv, cost F = 0.5 f^2 sum log1p((r/f)^2)
  camera step: R <- exp([dw]x) R (left perturbation), t <- t + dt; point X <- X + dX
  J_cam = J_Y [-[R X]x | I], J_pt = J_Y R (J_Y = d(u,v)/d(camera coords))
  g = sum w r J, H = sum wh J^T J with w = 1/(1+z), wh = max((1-z) w^2, 0.1 w)
  Marquardt damping on every diagonal; points eliminated by Schur complement:
    S = U + lam D_U - sum_i W_i (V_i + lam D_V)^-1 W_i^T ; b = -g_c + sum_i W_i M_i g_i
  accept iff F_new < F: lam /= 10 (>= LAM_MIN = 1e-7: the gauge is
  free, so lambda also keeps the reduced system non-singular); reject: lam *= 10
  stop: |g|_inf <= gtol | accept & (dF <= ftol F or |d| <= xtol (xtol + |x|)) | lam > 1e16
"""
import numpy as np

from .fisheye import project  # noqa: F401

LAM_MIN = 1e-7


def rodrigues(w):
    th = np.linalg.norm(w)
    if th < 1e-300:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.cos(th) * np.eye(3) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * Kx


def _skew(v):
    z = np.zeros(v.shape[:-1])
    return np.stack([np.stack([z, -v[..., 2], v[..., 1]], -1), np.stack([v[..., 2], z, -v[..., 0]], -1),
                     np.stack([-v[..., 1], v[..., 0], z], -1)], -2)


def _project_jy(Y, K, D):
    """Projection of camera-frame points Y (n,3) and d(u,v)/dY (n,2,3)."""
    fx, fy = K[..., 0, 0], K[..., 1, 1]
    d = D.reshape(D.shape[:-2] + (4,)) if D.shape[-1] == 1 else D
    iz = 1.0 / Y[:, 2]
    a = Y[:, 0] / Y[:, 2]
    b = Y[:, 1] / Y[:, 2]
    r2 = a * a + b * b
    r = np.sqrt(r2)
    th = np.arctan(r)
    th2 = th * th
    k1, k2, k3, k4 = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
    poly = 1 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4)))
    thd = th * poly
    dthd = 1 + th2 * (3 * k1 + th2 * (5 * k2 + th2 * (7 * k3 + th2 * 9 * k4)))
    big = r2 > 1e-16
    rs = np.where(big, r, 1.0)
    s = np.where(big, thd / rs, 1.0)
    spr = np.where(big, (dthd * rs / (1 + r2) - thd) / (rs ** 3), 0.0)
    u = fx * a * s + K[..., 0, 2]
    v = fy * b * s + K[..., 1, 2]
    duda, dudb = fx * (s + a * a * spr), fx * a * b * spr
    dvda, dvdb = fy * a * b * spr, fy * (s + b * b * spr)
    Ju = np.stack([duda * iz, dudb * iz, -(duda * a + dudb * b) * iz], -1)
    Jv = np.stack([dvda * iz, dvdb * iz, -(dvda * a + dvdb * b) * iz], -1)
    return np.stack([u, v], -1), np.stack([Ju, Jv], -2)


def residuals(X, R, t, K, D, uv, pi, ci):
    Y = np.einsum('nij,nj->ni', R[ci], X[pi]) + t[ci].reshape(-1, 3)
    p, _ = _project_jy(Y, K[ci], D[ci])
    return p - uv


def cost(X, R, t, K, D, uv, pi, ci, f):
    r = residuals(X, R, t, K, D, uv, pi, ci)
    return 0.5 * f * f * np.log1p(r * r / (f * f)).sum()


def linearize(X, R, t, K, D, uv, pi, ci, f_scale):
    """Cost, camera blocks U (C,6,6), g_c (C,6), point blocks V (n,3,3), g_p (n,3) and the
    per-observation coupling W (m,6,3) = J_cam^T wh J_pt, plus the raw Jacobians."""
    n, C = len(X), len(R)
    f2 = f_scale * f_scale
    RX = np.einsum('nij,nj->ni', R[ci], X[pi])
    Y = RX + t[ci]
    p, JY = _project_jy(Y, K[ci], D[ci])
    r = p - uv
    z = r * r / f2
    w = 1.0 / (1.0 + z)
    wh = np.maximum((1.0 - z) * w * w, 0.1 * w)
    Jp = JY @ R[ci]                                         # (m,2,3)
    Jc = np.concatenate([-JY @ _skew(RX), JY], -1)          # (m,2,6)
    F = 0.5 * f2 * np.log1p(z).sum()
    U = np.zeros((C, 6, 6))
    gc = np.zeros((C, 6))
    np.add.at(U, ci, np.einsum('md,mdi,mdj->mij', wh, Jc, Jc))
    np.add.at(gc, ci, np.einsum('md,md,mdi->mi', w, r, Jc))
    V = np.zeros((n, 3, 3))
    gp = np.zeros((n, 3))
    np.add.at(V, pi, np.einsum('md,mdi,mdj->mij', wh, Jp, Jp))
    np.add.at(gp, pi, np.einsum('md,md,mdi->mi', w, r, Jp))
    Wm = np.einsum('md,mdi,mdj->mij', wh, Jc, Jp)          # per observation (m,6,3)
    return F, U, gc, V, gp, Wm, Jc, Jp


def sba_extrinsics(points_2d, points_3d, point_idx, cam_idx, K, D, R0, t0, f_scale=1.0, max_iters=500,
                   ftol=1e-12, xtol=1e-12, gtol=1e-8, lam0=1e-3):
    uv = np.asarray(points_2d, np.float64)
    X = np.array(points_3d, np.float64).reshape(-1, 3)
    R = np.array(R0, np.float64).reshape(-1, 3, 3)
    t = np.array(t0, np.float64).reshape(-1, 3)
    K = np.asarray(K, np.float64)
    D = np.asarray(D, np.float64).reshape(-1, 4)
    pi = np.asarray(point_idx, np.int64)
    ci = np.asarray(cam_idx, np.int64)
    n, C = len(X), len(R)
    f2 = f_scale * f_scale

    def solve(U, gc, V, gp, Wm, lam):
        Ud = U.copy()
        Ud[:, range(6), range(6)] *= 1.0 + lam
        Vd = V.copy()
        Vd[:, range(3), range(3)] *= 1.0 + lam
        Vd[:, range(3), range(3)] += 1e-300
        M = np.linalg.inv(Vd)
        S = np.zeros((6 * C, 6 * C))
        for c in range(C):
            S[6 * c:6 * c + 6, 6 * c:6 * c + 6] += Ud[c]
        b = -gc.reshape(-1).copy()
        # Schur: per point, all pairs of its observations
        Z = np.einsum('mij,mjk->mik', Wm, M[pi])               # W_ci M_i (m,6,3)
        order = np.argsort(pi, kind='stable')
        starts = np.searchsorted(pi[order], np.arange(n + 1))
        for i in range(n):
            obs = order[starts[i]:starts[i + 1]]
            for o1 in obs:
                c1 = ci[o1]
                b[6 * c1:6 * c1 + 6] += Z[o1] @ gp[i]
                for o2 in obs:
                    c2 = ci[o2]
                    S[6 * c1:6 * c1 + 6, 6 * c2:6 * c2 + 6] -= Z[o1] @ Wm[o2].T
        dc = np.linalg.solve(S, b).reshape(C, 6)
        acc = gp.copy()
        np.add.at(acc, pi, np.einsum('mij,mi->mj', Wm, dc[ci]))
        dX = -np.einsum('nij,nj->ni', M, acc)
        return dc, dX

    F, U, gc, V, gp, Wm = linearize(X, R, t, K, D, uv, pi, ci, f_scale)[:6]
    F0, lam, status, iters, nacc = F, lam0, 'maxiter', 0, 0
    while iters < max_iters:
        gmax = max(np.abs(gc).max(), np.abs(gp).max())
        if gmax <= gtol:
            status = 'gtol'
            break
        dc, dX = solve(U, gc, V, gp, Wm, lam)
        Rn = np.array([rodrigues(dc[c, :3]) @ R[c] for c in range(C)])
        tn = t + dc[:, 3:]
        Xn = X + dX
        Fn = cost(Xn, Rn, tn, K, D, uv, pi, ci, f_scale)
        iters += 1
        dn = np.sqrt((dc ** 2).sum() + (dX ** 2).sum())
        xn = np.sqrt((t ** 2).sum() + (X ** 2).sum())
        if Fn < F:
            nacc += 1
            fconv = (F - Fn) <= ftol * abs(F)
            X, R, t = Xn, Rn, tn
            lam = max(lam * 0.1, LAM_MIN)
            F, U, gc, V, gp, Wm = linearize(X, R, t, K, D, uv, pi, ci, f_scale)[:6]
            if fconv:
                status = 'ftol'
                break
            if dn <= xtol * (xtol + xn):
                status = 'xtol'
                break
        else:
            lam *= 10.0
            if lam > 1e16:
                status = 'stalled'
                break
    return X, R, t, dict(status=status, iters=iters, n_accepted=nacc, cost_before=F0, cost_after=F, lam=lam)
