"""Oracle: Full Trajectory Estimation (FTE) objective and solver.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). **Parity unpinned against IPOPT**:
Pyomo, IPOPT and HSL MA86 are absent from this container and the reference ships no
FTE outputs, so this module restates the NLP of `src/core/fte.py:176-510` exactly and
minimises it with the same safeguarded Levenberg-Marquardt the GPU runs
(acinoset_amd/csrc/fte.hip); parity is GPU vs this oracle on identical inputs.

Reference NLP (src/core/fte.py), frames n = 1..N, cameras c, markers l, pose params p:
  poses[n,l]        = FK_l(x[n])                               (:323-328, misc.py:144)
  point[n,c,l]      = poses[n,l] + dx[n,0:3]*tau_c (+ ddx[n,0:3]*tau_c^2)   (:441-458)
  slack_meas        = proj_c(point) - meas                      (:460, proj :80-96)
  x[n]  = x[n-1]  + Ts*dx[n]      (n >= 2)                      (:467-471)
  dx[n] = dx[n-1] + Ts*ddx[n]     (n >= 2)                      (:473-477)
  ddx[n] = ddx[n-1] + slack_model[n]   (n >= 2)                 (:479-483)
  min  sum_{n,p} slack_model^2 / Q_p  +  sum redescending_loss(w_ncl * slack_meas, 3, 10, 20)
       Q_p = _Q[p]^2 (:113-144), w = 1/R = 1/3 if likelihood > thresh else 0 (:210-215)
  tau_1 = 0, -Ts <= tau_c <= Ts (const shutter-delay mode, :304-318)
  variable mode (:237-238, :307-314, :449-450): tau[n, c] per frame, tau[n, 1] = 0,
       -Ts <= tau[n, c] <= Ts, frame n's shift uses tau[n, c]

Exact elimination (no penalty, no approximation): with two virtual frames x[-1], x[0]
in front of the sequence, dx[n] = (x[n]-x[n-1])/Ts and ddx[n] = (dx[n]-dx[n-1])/Ts hold
for every n (the free dx[1], ddx[1] of the reference map one-to-one onto the virtual
frames), slack_model[n] = (x[n] - 3x[n-1] + 3x[n-2] - x[n-3]) / Ts^2 for n >= 2, and
slack_model[1] (free, unconstrained) is 0 at any optimum. Unknowns: X (N+2, P) + tau (C)
(const) or tau (N, C) (variable; flattened frame-major after X).

LM spec (shared with the GPU):
  H = sum_meas max(rho''(e), rho'(e)/e, 0) w^2 dproj^T dproj + 2 D^T diag(qinv) D (model, exact)
  g = sum_meas rho'(e) w dproj + 2 D^T diag(qinv) D X
  A = H + lam * diag(max(H_ii, 1e-12)); solve A d = -g (tau of camera 0 pinned, and every
      tau held at a bound whose -g points outward: active set, g zeroed there)
  trial: X + d_X, tau clipped to [-Ts, Ts]; accept iff F_new < F
  accept: lam = max(lam / 10, 1e-15); reject: lam *= 10
  stop: |g|_inf <= gtol | accept & (F - F_new <= ftol*|F| or |d| <= xtol*(xtol+|X|))
        | reject & lam > 1e16 | iters >= max_iters
"""
import numpy as np
import scipy.sparse as sp
import scipy.linalg as sla
import scipy.sparse.linalg as spla

from . import kinematics as okin
from .fisheye import project

INTERMODE = {'pos': 0, 'vel': 1, 'acc': 2}

# model-noise table of src/core/fte.py:113-143 (standard deviations; Q = value^2)
Q_TABLE = {'x_0': 4, 'y_0': 7, 'z_0': 5, 'phi_0': 13, 'theta_0': 9, 'psi_0': 26, 'l_1': 4, 'phi_1': 32,
           'theta_1': 18, 'psi_1': 12, 'theta_2': 43, 'phi_3': 10, 'theta_3': 53, 'psi_3': 34, 'theta_4': 90,
           'psi_4': 43, 'theta_5': 118, 'psi_5': 51, 'theta_6': 247, 'theta_7': 186, 'theta_8': 194,
           'theta_9': 164, 'theta_10': 295, 'theta_11': 243, 'theta_12': 334, 'theta_13': 149, 'x_l': 4,
           'y_l': 7, 'z_l': 5}


def qinv_for(mode):
    return np.array([1.0 / float(Q_TABLE[p]) ** 2 for p in okin.POSE[mode]])


class Problem:
    def __init__(self, mode, meas, w, K, D, R, t, Ts, sd=True, intermode='vel', a=3.0, b=10.0, c=20.0,
                 qinv=None, sd_mode='const'):
        self.mode = mode
        self.meas = np.nan_to_num(np.asarray(meas, np.float64))       # (N, C, L, 2)
        self.w = np.asarray(w, np.float64)                            # (N, C, L)
        self.meas[self.w == 0] = 0.0
        self.K, self.D, self.R, self.t = (np.asarray(v, np.float64) for v in (K, D, R, t))
        self.Ts = float(Ts)
        self.sd = bool(sd)
        self.im = INTERMODE[intermode] if sd else 0
        self.a, self.b, self.c = a, b, c
        self.N, self.C, self.L, _ = self.meas.shape
        self.P = len(okin.POSE[mode])
        self.M = self.N + 2
        self.qinv = qinv_for(mode) if qinv is None else np.asarray(qinv, np.float64)
        assert sd_mode in ('const', 'variable'), sd_mode
        self.var = sd_mode == 'variable' and self.sd
        self.tau_shape = (self.N, self.C) if self.var else (self.C,)
        self.nv = self.M * self.P + (int(np.prod(self.tau_shape)) if self.sd else 0)

    def tau_frames(self, tau):
        """(N, C) shutter delay of every frame (const mode: broadcast)."""
        tau = np.asarray(tau, np.float64)
        return tau if tau.ndim == 2 else np.broadcast_to(tau[None, :], (self.N, self.C))

    def pinned(self):
        """Indices of the unknowns fixed at 0: tau of camera 0 (src/core/fte.py:304-308)."""
        if not self.sd:
            return np.zeros(0, int)
        base = self.M * self.P
        return base + np.arange(self.N) * self.C if self.var else np.array([base])

    # ---- helpers --------------------------------------------------------------------
    def derivs(self, X):
        Ts = self.Ts
        x = X[2:]
        dx = (X[2:] - X[1:-1]) / Ts
        ddx = (X[2:] - 2 * X[1:-1] + X[:-2]) / (Ts * Ts)
        return x, dx, ddx

    def shift(self, X, tau):
        """(N, C, 3) shutter-delay shift of every marker."""
        if self.im == 0:
            return np.zeros((self.N, self.C, 3))
        _, dx, ddx = self.derivs(X)
        tf = self.tau_frames(tau)
        s = dx[:, None, :3] * tf[:, :, None]
        if self.im == 2:
            s = s + ddx[:, None, :3] * (tf ** 2)[:, :, None]
        return s

    def model_slack(self, X):
        return (X[3:] - 3 * X[2:-1] + 3 * X[1:-2] - X[:-3]) / (self.Ts * self.Ts)   # (N-1, P)

    def points(self, X, tau):
        pos = okin.marker_positions(self.mode, X[2:])                 # (N, L, 3)
        return pos[:, None, :, :] + self.shift(X, tau)[:, :, None, :]  # (N, C, L, 3)

    def residuals(self, X, tau):
        pts = self.points(X, tau)
        uv = np.empty(pts.shape[:-1] + (2,))
        for c in range(self.C):
            uv[:, c] = project(pts[:, c].reshape(-1, 3), self.K[c], self.D[c], self.R[c], self.t[c],
                               fte_form=True).reshape(self.N, self.L, 2)
        return self.w[..., None] * (uv - self.meas)                    # e (N, C, L, 2)

    def cost(self, X, tau, frames=None, stencils=None):
        """(total, measurement, model). `frames` (N,) / `stencils` (N-1,) boolean masks keep
        only those terms (the terms one rank owns in oracle/fte_dist.py)."""
        e = self.residuals(X, tau)
        rho = okin.redescending_loss(e, self.a, self.b, self.c)
        if frames is not None:
            rho = rho * np.asarray(frames, bool)[:, None, None, None]
        meas = rho.sum()
        s = self.model_slack(X)
        q = s * s * self.qinv
        if stencils is not None:
            q = q * np.asarray(stencils, bool)[:, None]
        model = q.sum()
        return meas + model, meas, model

    # ---- linearisation ----------------------------------------------------------------
    def linearize(self, X, tau, frames=None, stencils=None):
        """(cost, H, g) of the GN model; with masks, of the owned terms only (see cost)."""
        N, C, L, P, M, Ts = self.N, self.C, self.L, self.P, self.M, self.Ts
        fm = np.ones(N) if frames is None else np.asarray(frames, bool).astype(np.float64)
        x, dx, ddx = self.derivs(X)
        pos = okin.marker_positions(self.mode, x)                      # (N, L, 3)
        Jfk = okin.marker_jacobian(self.mode, x)                       # (N, L, 3, P)
        shift = self.shift(X, tau)
        tf = self.tau_frames(tau) if self.sd else np.zeros((N, C))
        rows, cols, vals = [], [], []
        grad = np.zeros(self.nv)
        F_meas = 0.0
        hcols = np.arange(P)
        for c in range(C):
            pt = pos + shift[:, c, None, :]
            uv, Jp = _project_jac_fte(pt.reshape(-1, 3), self.K[c], self.D[c], self.R[c], self.t[c])
            uv = uv.reshape(N, L, 2)
            Jp = Jp.reshape(N, L, 2, 3)
            e = self.w[:, c, :, None] * (uv - self.meas[:, c])          # (N, L, 2)
            rho = okin.redescending_loss(e, self.a, self.b, self.c)
            d1, d2 = okin.loss_derivs(e, self.a, self.b, self.c)
            F_meas += (rho * fm[:, None, None]).sum()
            wl = self.w[:, c, :, None] * fm[:, None, None]               # (N, L, 1)
            sq = np.sqrt(curvature(e, d1, d2)) * wl                      # scale of J rows
            gs = d1 * wl                                                 # scale of gradient rows
            # d proj / d x_k (own frame)
            Jown = np.einsum('nldk,nlkp->nldp', Jp, Jfk)                 # (N, L, 2, P)
            tc = tf[:, c, None, None, None]                              # (N, 1, 1, 1)
            a_own = a_prev = a_prev2 = 0.0
            if self.im >= 1:
                a_own += tc / Ts
                a_prev -= tc / Ts
            if self.im == 2:
                a_own += tc * tc / (Ts * Ts)
                a_prev -= 2 * tc * tc / (Ts * Ts)
                a_prev2 += tc * tc / (Ts * Ts)
            Jown[..., :3] += a_own * Jp
            blocks = [(0, Jown)]
            if self.im >= 1:
                blocks.append((-1, a_prev * Jp))
            if self.im == 2:
                blocks.append((-2, a_prev2 * Jp))
            ridx = (np.arange(N)[:, None, None] * C * L + c * L + np.arange(L)[None, :, None]) * 2 + \
                np.arange(2)[None, None, :]                               # residual row ids (N, L, 2)
            for off, Jb in blocks:
                width = Jb.shape[-1]
                f = np.arange(N) + 2 + off                               # frame index of this block
                colids = f[:, None, None, None] * P + np.arange(width)[None, None, None, :]
                colids = np.broadcast_to(colids, Jb.shape)
                rr = np.broadcast_to(ridx[..., None], Jb.shape)
                rows.append(rr.ravel())
                cols.append(colids.ravel())
                vals.append((Jb * sq[..., None]).ravel())
                np.add.at(grad, colids.ravel(), (Jb * gs[..., None]).ravel())
            if self.sd and c > 0:
                dtau = dx[:, :3] + (2 * tf[:, c, None] * ddx[:, :3] if self.im == 2 else 0.0)  # (N, 3)
                Jt = np.einsum('nldk,nk->nld', Jp, dtau)                 # (N, L, 2)
                colid = M * P + (np.arange(N) * C + c if self.var else np.full(N, c))
                colid = np.broadcast_to(colid[:, None, None], ridx.shape)
                rows.append(ridx.ravel())
                cols.append(colid.ravel())
                vals.append((Jt * sq).ravel())
                np.add.at(grad, colid.ravel(), (Jt * gs).ravel())
        Jm = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                           shape=(2 * N * C * L, self.nv))
        H = (Jm.T @ Jm).tocsr()
        # model term: slack_k = sum_i c_i X[k+3-i], c = [1, -3, 3, -1] / Ts^2 over frames k+3..k
        coef = np.array([1.0, -3.0, 3.0, -1.0]) / (Ts * Ts)
        s = self.model_slack(X)                                          # (N-1, P)
        nm = N - 1
        mrows, mcols, mvals = [], [], []
        for i, ci in enumerate(coef):
            f = np.arange(nm) + 3 - i
            mrows.append((np.arange(nm)[:, None] * P + hcols[None, :]).ravel())
            mcols.append((f[:, None] * P + hcols[None, :]).ravel())
            mvals.append(np.full(nm * P, ci))
        Dm = sp.csr_matrix((np.concatenate(mvals), (np.concatenate(mrows), np.concatenate(mcols))),
                           shape=(nm * P, self.nv))
        sm = np.ones(nm) if stencils is None else np.asarray(stencils, bool).astype(np.float64)
        qd = sp.diags(np.tile(self.qinv, nm) * np.repeat(sm, P))
        H = H + 2.0 * (Dm.T @ qd @ Dm)
        grad += 2.0 * (Dm.T @ (qd @ s.ravel()))
        F_model = float((s * s * self.qinv * sm[:, None]).sum())
        return F_meas + F_model, H.tocsr(), grad

    def pack(self, X, tau):
        return np.concatenate([X.ravel(), np.ravel(tau)]) if self.sd else X.ravel()

    def unpack(self, v):
        X = v[:self.M * self.P].reshape(self.M, self.P)
        tau = v[self.M * self.P:].reshape(self.tau_shape) if self.sd else np.zeros(self.tau_shape)
        return X, tau


def curvature(e, d1, d2):
    """GN curvature of the redescending loss: max(rho''(e), rho'(e)/e, 0). rho'/e is the
    IRLS majoriser weight (positive on the linear and redescending branches where
    rho'' <= 0); rho'' covers the cusp neighbourhood |e| < 0.06 where rho'/e < 0."""
    ae = np.abs(e)
    irls = np.where(ae > 1e-300, d1 / np.where(ae > 1e-300, e, 1.0), 0.0)
    return np.maximum(np.maximum(d2, irls), 0.0)


def _project_jac_fte(X, K, D, R, t):
    """FTE-form projection (r = sqrt(a^2+b^2+1e-12), src/core/fte.py:88) and d(u,v)/dX."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    d = np.asarray(D, np.float64).ravel()
    Y = X @ R.T + np.asarray(t).reshape(1, 3)
    iz = 1.0 / Y[:, 2]
    a = Y[:, 0] / Y[:, 2]
    b = Y[:, 1] / Y[:, 2]
    r = np.sqrt(a * a + b * b + 1e-12)
    th = np.arctan(r)
    th2 = th * th
    poly = 1 + th2 * (d[0] + th2 * (d[1] + th2 * (d[2] + th2 * d[3])))
    thd = th * poly
    dthd = 1 + th2 * (3 * d[0] + th2 * (5 * d[1] + th2 * (7 * d[2] + th2 * 9 * d[3])))
    s = thd / r
    spr = (dthd * r / (1 + r * r) - thd) / (r * r * r)
    u = fx * a * s + cx
    v = fy * b * s + cy
    duda, dudb = fx * (s + a * a * spr), fx * a * b * spr
    dvda, dvdb = fy * a * b * spr, fy * (s + b * b * spr)
    u0, u1, u2 = duda * iz, dudb * iz, -(duda * a + dudb * b) * iz
    v0, v1, v2 = dvda * iz, dvdb * iz, -(dvda * a + dvdb * b) * iz
    Ju = np.stack([u0, u1, u2], -1) @ R
    Jv = np.stack([v0, v1, v2], -1) @ R
    return np.stack([u, v], -1), np.stack([Ju, Jv], -2)


def active_bounds(prob, tau, g):
    """Shutter delays held at a bound of -Ts <= tau <= Ts whose descent direction -g
    points out of the box: pinned for this step (projected gradient / active set)."""
    t = np.ravel(tau)
    gt = g[prob.M * prob.P:]
    act = ((t >= prob.Ts) & (gt < 0)) | ((t <= -prob.Ts) & (gt > 0))
    return prob.M * prob.P + np.flatnonzero(act)


def _solve_step(prob, A, b):
    """Solve the damped normal equations A d = b (A SPD). Unknowns are ordered [X rows frame
    by frame | tau]. With a per-camera tau the X block is banded (a frame couples frames up
    to 3 away: half-bandwidth 4P - 1) with a C-column border, so it is a banded Cholesky
    (LAPACK pbtrf/pbtrs) plus a C x C Schur complement; with a per-frame tau (N*C border
    columns) a sparse LU."""
    if prob.var or not prob.sd:
        if not prob.sd:
            return sla.solveh_banded(_upper_band(A, prob.M * prob.P, 4 * prob.P - 1), b)
        return spla.spsolve(A, b)
    nx = prob.M * prob.P
    ab = _upper_band(A, nx, 4 * prob.P - 1)
    Axt = A[:nx, nx:].toarray()
    Z = sla.solveh_banded(ab, np.column_stack([b[:nx], Axt]))
    S = A[nx:, nx:].toarray() - Axt.T @ Z[:, 1:]
    dt = np.linalg.solve(S, b[nx:] - Axt.T @ Z[:, 0])
    return np.concatenate([Z[:, 0] - Z[:, 1:] @ dt, dt])


def _upper_band(A, n, u):
    """Upper band storage ab[u + i - j, j] = A[i, j] (i <= j) of A[:n, :n]."""
    c = A[:n, :n].tocoo()
    m = c.row <= c.col
    if m.any() and int((c.col[m] - c.row[m]).max()) > u:
        raise ValueError('normal matrix wider than the assumed time band')
    ab = np.zeros((u + 1, n))
    np.add.at(ab, (u + c.row[m] - c.col[m], c.col[m]), c.data[m])
    return ab


def solve(prob, X0, tau0=None, max_iters=200, ftol=1e-12, xtol=1e-12, gtol=1e-8, lam0=1e-3, verbose=False):
    """LM of the module docstring. Returns (X, tau, info). BLAS runs on one thread: the
    banded factorisation of a 104-wide band is 10x slower with a thread team (OpenBLAS)."""
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1, user_api='blas'):
        return _solve(prob, X0, tau0, max_iters, ftol, xtol, gtol, lam0, verbose)


def _solve(prob, X0, tau0, max_iters, ftol, xtol, gtol, lam0, verbose):
    X = np.array(X0, np.float64).reshape(prob.M, prob.P)
    tau = np.zeros(prob.tau_shape) if tau0 is None else np.array(tau0, np.float64).reshape(prob.tau_shape)
    tau[..., 0] = 0.0
    F, H, g = prob.linearize(X, tau)
    F0 = F
    lam = lam0
    status, iters, n_acc = 'maxiter', 0, 0
    pin0 = prob.pinned() if prob.sd else None
    pin = pin0
    while iters < max_iters:
        gp = g
        if pin0 is not None:
            # the active set comes from the true gradient at the current state; the pinned
            # (projected) copy drives the step, so a rejected step leaves g untouched
            pin = np.concatenate([pin0, active_bounds(prob, tau, g)])
            gp = g.copy()
            gp[pin] = 0.0
        gmax = float(np.abs(gp).max())
        if gmax <= gtol:
            status = 'gtol'
            break
        dg = H.diagonal()
        A = (H + sp.diags(lam * np.maximum(dg, 1e-12))).tocsc()
        if pin is not None:
            # pinned unknowns: their rows and columns replaced by the identity (a diagonal
            # mask on both sides, so the matrix stays in CSC)
            keep = np.ones(prob.nv)
            keep[pin] = 0.0
            A = (sp.diags(keep) @ A @ sp.diags(keep) + sp.diags(1.0 - keep)).tocsc()
        d = _solve_step(prob, A, -gp)
        dX, dtau = prob.unpack(d)
        Xn = X + dX
        taun = np.clip(tau + dtau, -prob.Ts, prob.Ts) if prob.sd else tau
        if prob.sd:
            taun[..., 0] = 0.0
        Fn = prob.cost(Xn, taun)[0]
        iters += 1
        xn = np.linalg.norm(prob.pack(X, tau))
        small = np.linalg.norm(d) <= xtol * (xtol + xn)
        if Fn < F:
            n_acc += 1
            fconv = (F - Fn) <= ftol * abs(F)
            X, tau = Xn, taun
            lam = max(lam * 0.1, 1e-15)
            F, H, g = prob.linearize(X, tau)
            if verbose:
                print(f'it {iters:3d} F {F:.10e} lam {lam:.1e} |d| {np.linalg.norm(d):.3e}')
            if fconv:
                status = 'ftol'
                break
            if small:
                status = 'xtol'
                break
        else:
            lam *= 10.0
            if lam > 1e16:
                status = 'stalled'
                break
    Fm = prob.cost(X, tau)
    return X, tau, dict(status=status, iters=iters, n_accepted=n_acc, cost_before=F0, cost_after=Fm[0],
                        cost_meas=Fm[1], cost_model=Fm[2], lam=lam)


def initial_state(prob, nose_frames, nose_xyz, start_frame=0):
    """FTE init of src/core/fte.py:254-292: linear regression of the triangulated nose
    over absolute frame numbers -> x_0, y_0, z_0; psi_0 = atan2(y_slope, x_slope); all
    other parameters 0; dx = ddx = 0 (virtual frames = first frame)."""
    from scipy.stats import linregress
    idx = {k: i for i, k in enumerate(okin.POSE[prob.mode])}
    fr = np.asarray(nose_frames, np.float64)
    sx, ix = linregress(fr, nose_xyz[:, 0])[:2]
    sy, iy = linregress(fr, nose_xyz[:, 1])[:2]
    sz, iz = linregress(fr, nose_xyz[:, 2])[:2]
    f = np.arange(start_frame, start_frame + prob.N)
    x = np.zeros((prob.N, prob.P))
    x[:, idx['x_0']] = f * sx + ix
    x[:, idx['y_0']] = f * sy + iy
    x[:, idx['z_0']] = f * sz + iz
    x[:, idx['psi_0']] = np.arctan2(sy, sx)
    X = np.concatenate([x[:1], x[:1], x], 0)
    return X
