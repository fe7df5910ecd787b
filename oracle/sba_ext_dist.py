"""Oracle: points + extrinsics SBA split over ranks.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Spec of acs_sba_ext_dist_* (acinoset_amd/csrc/sba_ext.hip) restated with
numpy on top of oracle/sba_ext.py: each rank holds a contiguous shard of the points and
their observations, the cameras are replicated.

* payload 1 (summed over ranks): the rank's Schur complement of its points on the camera
  system, undamped: S_r = blockdiag(U_r) - sum_i W_i M_i W_i^T, b_r = -g_c,r + sum_i W_i M_i
  g_i with M_i = (V_i + lam diag V_i)^-1, plus diag U_r, g_c,r and max |g_p| over its points;
* every rank damps S = sum S_r with lam * max(diag U, 1e-12), solves for the camera step,
  steps its own points, and puts (cost, |dX|^2, |X|^2) of its points into payload 3;
* the accept/reject rule and the damping floor are oracle/sba_ext.py's.

Round protocol (one all-reduce per LM step, acs_sba_ext_dist_round): the payload is
[p1 | p3]. init() gives the starting state's system and cost; round(P) decides on the
pending trial from P's p3, steps from P's p1, and returns the next payload: the trial's p3
and the system at the trial state with the damping an acceptance sets (speculation). A
rejection skips the step and re-forms the system at the current state (one extra round).
poll(k) is the status after round k.
"""
import numpy as np

from . import sba_ext as ose


class OracleSbaExtRank:
    def __init__(self, points_2d, points_3d, point_idx, cam_idx, K, D, R0, t0, rank=0, world=1, f_scale=1.0,
                 max_iters=500, ftol=1e-12, xtol=1e-12, gtol=1e-8, lam0=1e-3):
        self.uv = np.asarray(points_2d, np.float64).reshape(-1, 2)
        self.X = np.array(points_3d, np.float64).reshape(-1, 3)
        self.pi = np.asarray(point_idx, np.int64)
        self.ci = np.asarray(cam_idx, np.int64)
        self.K = np.asarray(K, np.float64)
        self.D = np.asarray(D, np.float64).reshape(-1, 4)
        self.R = np.array(R0, np.float64).reshape(-1, 3, 3)
        self.t = np.array(t0, np.float64).reshape(-1, 3)
        self.rank, self.world, self.f = rank, world, f_scale
        self.opts = dict(max_iters=max_iters, ftol=ftol, xtol=xtol, gtol=gtol)
        self.lam, self.status, self.iters, self.nacc, self.relin = lam0, 0, 0, 0, True
        self.C = len(self.R)

    def _cost(self, X, R, t):
        return ose.cost(X, R, t, self.K, self.D, self.uv, self.pi, self.ci, self.f)

    def init(self):
        self.first, self.pending, self.rounds = True, False, []
        p3 = np.array([self._cost(self.X, self.R, self.t), 0.0, 0.0])
        return np.concatenate([self.phase1(), p3])

    def _decide(self, p3):
        """k_ext_decide: the pending trial kept or discarded; True = skip this round's step."""
        if self.first:
            self.first = False
            self.F = self.F0 = float(p3[0])
            if self.opts['max_iters'] <= 0:       # no step at all
                self.status = 5
            return False
        if self.status or not self.pending:
            return False
        self.pending = False
        self.phase3(p3)
        return self.status == 0 and not self.relin

    def round(self, P):
        n1 = len(P) - 3
        skip = self._decide(P[n1:])
        out = np.zeros_like(P)
        if self.status == 0 and not skip:
            out[n1:] = self.phase2(P[:n1])
            self.pending = True
            # the next system at the trial state, with an acceptance's damping
            keep = (self.X, self.R, self.t, self.lam)
            self.X, self.R, self.t = self.Xn, self.Rn, self.tn
            self.lam = max(self.lam * 0.1, ose.LAM_MIN)
            self.relin = True
            out[:n1] = self.phase1()
            self.X, self.R, self.t, self.lam = keep
        elif self.status == 0:
            self.relin = True            # the speculative system replaced this state's linearisation
            out[:n1] = self.phase1()
        self.rounds.append(self.status)
        return out

    def poll(self, k):
        return self.rounds[k]

    def phase1(self):
        C, n = self.C, len(self.X)
        if self.relin:
            (self.Fl, self.U, self.gc, self.V, self.gp,
             self.Wm) = ose.linearize(self.X, self.R, self.t, self.K, self.D, self.uv, self.pi, self.ci, self.f)[:6]
        Vd = self.V.copy()
        Vd[:, range(3), range(3)] *= 1.0 + self.lam
        Vd[:, range(3), range(3)] += 1e-300
        self.M = np.linalg.inv(Vd) if n else np.zeros((0, 3, 3))
        S = np.zeros((6 * C, 6 * C))
        for c in range(C):
            S[6 * c:6 * c + 6, 6 * c:6 * c + 6] += self.U[c]
        b = -self.gc.reshape(-1).copy()
        Z = np.einsum('mij,mjk->mik', self.Wm, self.M[self.pi])
        for i in range(n):
            obs = np.nonzero(self.pi == i)[0]
            for o1 in obs:
                c1 = self.ci[o1]
                b[6 * c1:6 * c1 + 6] += Z[o1] @ self.gp[i]
                for o2 in obs:
                    c2 = self.ci[o2]
                    S[6 * c1:6 * c1 + 6, 6 * c2:6 * c2 + 6] -= Z[o1] @ self.Wm[o2].T
        out = np.zeros(36 * C * C + 18 * C + self.world)
        NC = 6 * C
        out[:NC * NC] = S.ravel()
        out[NC * NC:NC * NC + NC] = b
        out[NC * NC + NC:NC * NC + 2 * NC] = np.stack([np.diag(u) for u in self.U]).ravel()
        out[NC * NC + 2 * NC:NC * NC + 3 * NC] = self.gc.ravel()
        out[NC * NC + 3 * NC + self.rank] = np.abs(self.gp).max() if n else 0.0
        return out

    def phase2(self, p1):
        C = self.C
        NC = 6 * C
        S = p1[:NC * NC].reshape(NC, NC).copy()
        b = p1[NC * NC:NC * NC + NC]
        udiag = p1[NC * NC + NC:NC * NC + 2 * NC]
        gc = p1[NC * NC + 2 * NC:NC * NC + 3 * NC]
        self.gmax = max(np.abs(gc).max(), p1[NC * NC + 3 * NC:].max())
        S[np.diag_indices_from(S)] += self.lam * np.maximum(udiag, 1e-12)
        dc = np.linalg.solve(S, b).reshape(C, 6)
        acc = self.gp.copy()
        np.add.at(acc, self.pi, np.einsum('mij,mi->mj', self.Wm, dc[self.ci]))
        dX = -np.einsum('nij,nj->ni', self.M, acc)
        self.Rn = np.array([ose.rodrigues(dc[c, :3]) @ self.R[c] for c in range(C)])
        self.tn = self.t + dc[:, 3:]
        self.Xn = self.X + dX
        self.dcn = (dc ** 2).sum()
        return np.array([self._cost(self.Xn, self.Rn, self.tn), (dX ** 2).sum(), (self.X ** 2).sum()])

    def phase3(self, p3, init=False):
        o = self.opts
        if init:
            self.F = self.F0 = float(p3[0])
            return 0
        if self.status:
            return self.status
        if self.gmax <= o['gtol']:
            self.status = 1
            return 1
        Fn = float(p3[0])
        self.iters += 1
        dn = np.sqrt(p3[1] + self.dcn)
        xn = np.sqrt(p3[2] + (self.t ** 2).sum())
        if Fn < self.F:
            fconv = (self.F - Fn) <= o['ftol'] * abs(self.F)
            self.nacc += 1
            self.F = Fn
            self.X, self.R, self.t = self.Xn, self.Rn, self.tn
            self.lam = max(self.lam * 0.1, ose.LAM_MIN)
            self.relin = True
            if fconv:
                self.status = 2
            elif dn <= o['xtol'] * (o['xtol'] + xn):
                self.status = 3
        else:
            self.lam *= 10.0
            self.relin = False
            if self.lam > 1e16:
                self.status = 4
        if self.status == 0 and self.iters >= o['max_iters']:
            self.status = 5
        return self.status

    def result(self):
        return self.R, self.t, self.X, dict(status=self.status, iters=self.iters, n_accepted=self.nacc,
                                            cost_before=self.F0, cost_after=self.F, lam=self.lam)
