"""The algebraic identities the EKF kernels rest on (csrc/ekf.hip), checked in float64 numpy
on random well-conditioned instances - CPU only. The kernels' parity against the oracle is in
tests/test_gpu_ekf.py; these pin that the reformulations are exact, not approximations:

  * the Woodbury update in SPD form: (I + A C)^-1 = W^-1 C with W = C + C A C (both filters),
    and its guard: diagonal pivots are used only while every pivot is positive (W > 0), and
    the reference's default P0 (src/core/ekf.py:155, a -0.28 variance) takes the partially
    pivoted solve of [I + A C | I] instead;
  * the analytic H in marker space: H^T W H = sum_l D_l^T M_l D_l, H^T W r = sum_l D_l^T g_l
    and diag(H C H^T)_r = j_r N_l j_r^T (k_ekf_filter<*, true>);
  * the RTS gain as a solve: A_i^T = P_pred^-1 (P_est F^T)^T (k_ekf_gain_w, src/core/ekf.py:294).
"""
import numpy as np

from oracle import ekf as oekf


def _spd(rng, n, scale=1.0):
    a = rng.standard_normal((n, n))
    return scale * (a @ a.T / n + 0.5 * np.eye(n))


def test_woodbury_spd_form():
    rng = np.random.default_rng(0)
    for P in (6, 29):
        C = _spd(rng, P, 1e-2)
        Hx = rng.standard_normal((4 * P, P)) * 300.0
        w = 1.0 / rng.uniform(1.0, 9.0, 4 * P)
        A = Hx.T @ (w[:, None] * Hx)
        M = np.eye(P) + A @ C
        W = C + C @ A @ C
        np.testing.assert_allclose(W, W.T, rtol=1e-12, atol=0)
        assert np.all(np.linalg.eigvalsh(W) > 0)
        V = np.linalg.solve(W, C)
        np.testing.assert_allclose(V, np.linalg.inv(M), rtol=1e-8, atol=1e-12)
        # the update it feeds: (I + A C)^-1 A = V A, symmetric
        Y = V @ A
        np.testing.assert_allclose(Y, Y.T, rtol=1e-7, atol=1e-9 * np.abs(Y).max())


def test_marker_space_analytic_h():
    rng = np.random.default_rng(1)
    P, L, Cn = 29, 21, 12
    D = rng.standard_normal((L, 3, P))             # d pos_l / d x
    J = rng.standard_normal((Cn, L, 2, 3)) * 400   # projection Jacobians (rows u, v)
    w = 1.0 / rng.uniform(1.0, 9.0, (Cn, L, 2))    # R^-1
    r = rng.standard_normal((Cn, L, 2))
    Cxx = _spd(rng, P, 1e-2)
    # row form: H row (c, l, side) = J[c, l, side] @ D[l]
    H = np.einsum('clsk,lkp->clsp', J, D).reshape(-1, P)
    wf, rf = w.reshape(-1), r.reshape(-1)
    A_rows = H.T @ (wf[:, None] * H)
    b_rows = H.T @ (wf * rf)
    q_rows = np.einsum('ip,pq,iq->i', H, Cxx, H)
    # marker space: M_l = sum_c J^T W J, g_l = sum_c J^T W r, N_l = D_l C D_l^T
    M = np.einsum('clsa,cls,clsb->lab', J, w, J)
    g = np.einsum('clsa,cls,cls->la', J, w, r)
    A_mk = np.einsum('lap,lab,lbq->pq', D, M, D)
    b_mk = np.einsum('lap,la->p', D, g)
    N = np.einsum('lap,pq,lbq->lab', D, Cxx, D)
    q_mk = np.einsum('clsa,lab,clsb->cls', J, N, J).reshape(-1)
    np.testing.assert_allclose(A_mk, A_rows, rtol=1e-10, atol=1e-10 * np.abs(A_rows).max())
    np.testing.assert_allclose(b_mk, b_rows, rtol=1e-10, atol=1e-10 * np.abs(b_rows).max())
    np.testing.assert_allclose(q_mk, q_rows, rtol=1e-10, atol=0)


def test_rts_gain_as_spd_solve():
    rng = np.random.default_rng(2)
    P = 6
    n = 3 * P
    sT = 1 / 90.0
    F = oekf.transition(P, sT)
    Pe = _spd(rng, n, 1e-2)
    Pp = F @ Pe @ F.T + _spd(rng, n, 1e-4)
    A_ref = Pe @ F.T @ np.linalg.inv(Pp)             # src/core/ekf.py:294
    At = np.linalg.solve(Pp, (Pe @ F.T).T)           # k_ekf_gain_w: P_pred^-1 (P_est F^T)^T
    np.testing.assert_allclose(At.T, A_ref, rtol=1e-9, atol=1e-12 * np.abs(A_ref).max())


def _gj_diag(W, C):
    """k_ekf_filter's diagonal-pivot Gauss-Jordan on [W | C] (row k is pivot k); returns
    (V, ok) where ok is False at the first pivot that is not positive (the kernel then
    switches to _gj_pivoted)."""
    P = W.shape[0]
    a = np.hstack([W, C]).astype(float)
    for k in range(P):
        p = a[k, k]
        if not p > 0:
            return None, False
        f = a[:, k] / p
        f[k] = 0.0
        a[:, k + 1:] -= np.outer(f, a[k, k + 1:])
    return a[:, P:] / np.diag(a)[:, None], True


def _gj_pivoted(M):
    """ekf_update_pivoted / ekf_w1_pivoted: Gauss-Jordan with implicit partial pivoting on
    [M | I] (largest |a[r][k]| among the unused rows, lowest row on ties); row pv_k over its
    pivot is row k of M^-1."""
    P = M.shape[0]
    a = np.hstack([M, np.eye(P)])
    used = np.zeros(P, bool)
    V = np.zeros((P, P))
    piv = []
    for k in range(P):
        col = np.where(used, -1.0, np.abs(a[:, k]))
        pv = int(np.argmax(col))            # first maximum: lowest row on ties
        p = a[pv, k]
        f = a[:, k] / p
        f[pv] = 0.0
        a[:, k + 1:] -= np.outer(f, a[pv, k + 1:])
        used[pv] = True
        piv.append((pv, p))
    for k, (pv, p) in enumerate(piv):
        V[k] = a[pv, P:] / p
    return V


def test_woodbury_default_p0_is_indefinite_and_takes_the_pivoted_solve():
    """the default model's P0 has a -0.28 neck-length variance, so P_xx and W are
    indefinite; with low-likelihood frames (R = maxpix^2, A tiny) or a weakly observed neck a
    leading minor of W passes through zero. The kernels certify W > 0 by its pivots and else
    solve I + A C with partial pivoting, which matches inv(I + A C) in every case here."""
    rng = np.random.default_rng(4)
    P = 29
    sT = 1 / 90.0
    F = oekf.transition(P, sT)
    Pp = F @ oekf.initial_covariance('default') @ F.T + oekf.process_noise(P, sT)
    C = Pp[:P, :P]
    assert np.linalg.eigvalsh(C).min() < -0.2
    for wscale in (1.0, 1.0 / 2704.0 ** 2, 1e-12):      # good, low-likelihood, unobserved
        Hx = rng.standard_normal((8 * P, P)) * 300.0
        Hx[:, 6] *= 1e-3                                  # neck length weakly observed
        w = wscale / rng.uniform(1.0, 9.0, 8 * P)
        A = Hx.T @ (w[:, None] * Hx)
        M = np.eye(P) + A @ C
        W = C + C @ A @ C
        assert np.linalg.eigvalsh(W).min() < 0            # W is not positive definite
        _, ok = _gj_diag(W, C)
        assert not ok                                     # the pivot check sees it
        V = _gj_pivoted(M)
        np.testing.assert_allclose(V @ M, np.eye(P), atol=1e-9)
        np.testing.assert_allclose(V, np.linalg.inv(M), rtol=1e-7, atol=1e-10 * np.abs(V).max())
    # a leading minor of W near zero with W nonsingular (eigenvalues +-1): the first pivot is
    # a tiny positive 1e-17, the second -1e17, so the check rejects the diagonal solve before
    # its result is used, and the pivoted solve of the same system is exact
    W2 = np.array([[1e-17, 1.0], [1.0, 1e-17]])
    _, ok = _gj_diag(W2, np.eye(2))
    assert not ok
    np.testing.assert_allclose(_gj_pivoted(W2) @ W2, np.eye(2), atol=1e-15)


def test_woodbury_spd_case_keeps_the_diagonal_solve():
    """The head model's P0 is positive definite: every pivot is positive and the diagonal
    solve equals inv(I + A C)."""
    rng = np.random.default_rng(5)
    P = 6
    sT = 1 / 90.0
    F = oekf.transition(P, sT)
    Pp = F @ oekf.initial_covariance('head') @ F.T + oekf.process_noise(P, sT)
    C = Pp[:P, :P]
    Hx = rng.standard_normal((24 * P, P)) * 300.0
    w = 1.0 / rng.uniform(1.0, 9.0, 24 * P)
    A = Hx.T @ (w[:, None] * Hx)
    V, ok = _gj_diag(C + C @ A @ C, C)
    assert ok
    np.testing.assert_allclose(V, np.linalg.inv(np.eye(P) + A @ C), rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(_gj_pivoted(np.eye(P) + A @ C), V, rtol=1e-7, atol=1e-12)
