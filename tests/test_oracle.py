"""CPU: pin the oracle (and the product's skeleton tables) to the reference's own
outputs captured in tests/golden/ (see tests/golden/make_golden.py)."""
import numpy as np
import pytest

from conftest import golden
from oracle import fisheye, kinematics as okin, sba as osba
from acinoset_amd import kinematics as pkin


def _shift(g, mode, inter):
    dx, ddx, tau = g[f'{mode}_dx'], g[f'{mode}_ddx'], g[f'{mode}_tau']
    if inter == 'pos':
        return None
    s = dx[:, :3] * tau[:, None]
    if inter == 'acc':
        s = s + ddx[:, :3] * (tau ** 2)[:, None]
    return s


@pytest.mark.parametrize('mode', ['default', 'head', 'upper_body', 'head_stabilize'])
@pytest.mark.parametrize('inter', ['pos', 'vel', 'acc'])
@pytest.mark.parametrize('dirs', [0, 1])
def test_oracle_fk_matches_reference(mode, inter, dirs):
    g = golden('fk')
    ref = g[f'{mode}_{inter}_{dirs}']
    out = okin.marker_positions(mode, g[f'{mode}_x'], _shift(g, mode, inter), directions=bool(dirs))
    if mode == 'default':
        # the reference never shifts the lure (src/lib/misc.py:222)
        out[:, 20] = g['default_x'][:, 26:29]
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12)


@pytest.mark.parametrize('mode', ['default', 'head', 'upper_body', 'head_stabilize'])
@pytest.mark.parametrize('inter', ['pos', 'vel', 'acc'])
def test_table_fk_matches_reference(mode, inter):
    """The product's skeleton *table* (what the HIP kernel evaluates) reproduces the
    reference FK (host evaluation of the table)."""
    g = golden('fk')
    ref = g[f'{mode}_{inter}_1']
    out = pkin.fk_numpy(mode, g[f'{mode}_x'], _shift(g, mode, inter), directions=True)
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12)


def test_table_jacobian_structure_matches_complex_step():
    """Host check of the analytic-Jacobian tables (deriv mask) against complex step."""
    rng = np.random.default_rng(0)
    for mode in ('default', 'default_nolure', 'head', 'upper_body', 'head_stabilize'):
        t = pkin.build_table(mode)
        x = rng.normal(0, 0.4, (3, t.P))
        J = okin.marker_jacobian(mode, x)                 # (n, L, 3, P)
        nz = (np.abs(J) > 1e-14).any(axis=(0, 2))           # (L, P)
        K = t.n_nodes
        deriv = t.ints[-K * t.P:].reshape(K, t.P)
        J_ = t.n_joints
        off = pkin.INT_HDR + 9 * J_ + 4 * K
        outn = t.ints[off:off + t.L]
        assert np.all(deriv[outn].astype(bool) >= nz), mode  # mask covers every true dependency


def test_loss_matches_reference():
    g = golden('loss')
    np.testing.assert_allclose(okin.redescending_loss(g['err']), g['loss'], rtol=1e-14, atol=1e-14)


def test_loss_derivatives_fd():
    e = np.concatenate([np.linspace(-25, -0.01, 400), np.linspace(0.01, 25, 400)])
    h = 1e-6
    d1, d2 = okin.loss_derivs(e)
    fd1 = (okin.redescending_loss(e + h) - okin.redescending_loss(e - h)) / (2 * h)
    fd2 = (okin.loss_derivs(e + h)[0] - okin.loss_derivs(e - h)[0]) / (2 * h)
    np.testing.assert_allclose(d1, fd1, atol=1e-7)
    np.testing.assert_allclose(d2, fd2, atol=1e-6)


def test_projection_jacobian_fd():
    g = golden('sba_cfg2')
    rng = np.random.default_rng(1)
    X = g['points_3d'][:50] + rng.normal(0, 0.1, (50, 3))
    ci = rng.integers(0, 6, 50)
    uv, J = fisheye.project_jac(X, g['K'][ci], g['D'][ci], g['R'][ci], g['t'][ci])
    np.testing.assert_allclose(uv, fisheye.project(X, g['K'][ci], g['D'][ci], g['R'][ci], g['t'][ci]), atol=1e-9)
    h = 1e-6
    for k in range(3):
        e = np.zeros(3)
        e[k] = h
        fd = (fisheye.project(X + e, g['K'][ci], g['D'][ci], g['R'][ci], g['t'][ci])
              - fisheye.project(X - e, g['K'][ci], g['D'][ci], g['R'][ci], g['t'][ci])) / (2 * h)
        np.testing.assert_allclose(J[..., k], fd, rtol=1e-6, atol=1e-4)


@pytest.mark.parametrize('name', ['sba_cfg1', 'sba_cfg2'])
def test_oracle_sba_matches_reference(name):
    g = golden(name)
    n = len(g['points_3d'])
    # residuals['before'] (reference cost function at the reference init)
    f0 = osba.cost_func_points_only(g['points_3d'].ravel(), n, g['point_indices'], g['camera_indices'],
                                    g['K'], g['D'], g['R'], g['t'], g['points_2d'])
    np.testing.assert_allclose(f0, g['resid_before'], rtol=0, atol=1e-9)
    x, info = osba.sba_points(g['points_2d'], g['points_3d'], g['point_indices'], g['camera_indices'],
                              g['K'], g['D'], g['R'], g['t'], return_info=True)
    d = np.linalg.norm(x - g['pts_out'], axis=1)
    # scipy stops on xtol=1e-8 (relative); the oracle converges tighter. Contract: 1e-4 m RMS.
    assert np.sqrt(np.mean(d ** 2)) < 1e-6 and d.max() < 1e-5
    assert np.all(info['cost_after'] <= info['cost_before'] + 1e-9)
    f1 = osba.cost_func_points_only(x.ravel(), n, g['point_indices'], g['camera_indices'],
                                    g['K'], g['D'], g['R'], g['t'], g['points_2d'])
    np.testing.assert_allclose(f1, g['resid_after'], atol=1e-3)
    # robust cost no larger than the reference's
    c_ref = 0.5 * 2500 * np.log1p(g['resid_after'] ** 2 / 2500).sum()
    assert 0.5 * 2500 * np.log1p(f1 ** 2 / 2500).sum() <= c_ref + 1e-9


def test_oracle_triangulation_matches_reference():
    g = golden('triangulation')
    X = fisheye.triangulate_pair(g['pair_a'], g['pair_b'], g['K'][0], g['D'][0], g['R'][0], g['t'][0],
                                 g['K'][1], g['D'][1], g['R'][1], g['t'][1])
    np.testing.assert_allclose(X, g['pair_xyz'], atol=1e-9)
    fr, mk, xyz = fisheye.pairwise_points(g['df_frame'], g['df_camera'], g['df_marker'], g['df_x'], g['df_y'],
                                          g['K'], g['D'], g['R'], g['t'])
    ref = {(f, m): p for f, m, p in zip(g['out_frame'], g['out_marker'], g['out_xyz'])}
    assert len(ref) == len(fr)
    for f, m, p in zip(fr, mk, xyz):
        np.testing.assert_allclose(p, ref[(f, m)], atol=1e-9)


def _ext_args(g):
    return (g['K'], g['D'].reshape(-1, 4), g['points_2d'], g['point_indices'].astype(np.int64),
            g['camera_indices'].astype(np.int64))


def test_oracle_sba_extrinsics_cost_matches_reference():
    """Golden `bundle_adjust_points_and_extrinsics` (src/lib/sba.py:158-178): the oracle's
    residual function reproduces the reference's before/after residual vectors at the
    reference's own initial and final states."""
    from oracle import sba_ext
    g = golden('sba_extrinsics')
    K, D, uv, pi, ci = _ext_args(g)
    r0 = sba_ext.residuals(g['points_3d'], g['R0'], g['t0'].reshape(-1, 3), K, D, uv, pi, ci)
    np.testing.assert_allclose(r0.ravel(), g['resid_before'], atol=1e-9)
    r1 = sba_ext.residuals(g['obj_out'], g['R_out'], g['t_out'].reshape(-1, 3), K, D, uv, pi, ci)
    np.testing.assert_allclose(r1.ravel(), g['resid_after'], atol=1e-6)


def test_oracle_sba_extrinsics_jacobian_fd():
    """Left-perturbation camera Jacobian [-J_Y [R X]x | J_Y] and point Jacobian J_Y R vs
    central differences of the residual function."""
    from oracle import sba_ext
    g = golden('sba_extrinsics')
    K, D, uv, pi, ci = _ext_args(g)
    X, R, t = g['points_3d'], g['R0'], g['t0'].reshape(-1, 3)
    *_, Jc, Jp = sba_ext.linearize(X, R, t, K, D, uv, pi, ci, 1.0)
    h = 1e-6
    for k in range(6):
        c = 2
        dw = np.zeros(6)
        dw[k] = h
        def res(s):
            Rn, tn = R.copy(), t.copy()
            Rn[c] = sba_ext.rodrigues(s * dw[:3]) @ R[c]
            tn[c] = t[c] + s * dw[3:]
            return sba_ext.residuals(X, Rn, tn, K, D, uv, pi, ci)
        fd = (res(1) - res(-1)) / (2 * h)
        sel = ci == c
        np.testing.assert_allclose(Jc[sel, :, k], fd[sel], rtol=1e-5, atol=1e-3)
    for k in range(3):
        e = np.zeros(3)
        e[k] = h
        fd = (sba_ext.residuals(X + e, R, t, K, D, uv, pi, ci) - sba_ext.residuals(X - e, R, t, K, D, uv, pi, ci)) / (
            2 * h)
        np.testing.assert_allclose(Jp[..., k], fd, rtol=1e-5, atol=1e-3)


def test_oracle_sba_extrinsics_beats_reference_cost():
    """Parity on the objective (scipy stopped unconverged): the oracle's
    Schur LM reaches a robust cost no larger than the reference's final state."""
    from oracle import sba_ext
    g = golden('sba_extrinsics')
    K, D, uv, pi, ci = _ext_args(g)
    X, R, t, info = sba_ext.sba_extrinsics(uv, g['points_3d'], pi, ci, K, D, g['R0'], g['t0'], max_iters=200)
    c_ref = 0.5 * np.log1p(g['resid_after'] ** 2).sum()
    c0 = 0.5 * np.log1p(g['resid_before'] ** 2).sum()
    assert abs(info['cost_before'] - c0) < 1e-9 * c0
    assert info['cost_after'] <= c_ref
    np.testing.assert_allclose(R @ np.swapaxes(R, 1, 2), np.broadcast_to(np.eye(3), R.shape), atol=1e-12)


def _ekf_golden(mode):
    from oracle import ekf as oekf
    g = golden(f'ekf_{mode}')
    N = int(g['n_frames'])
    uv, lik = g['uv'], g['likelihood']
    C, L = uv.shape[1], uv.shape[2]
    fr, ca, mk = np.meshgrid(np.arange(N), np.arange(C), np.arange(L), indexing='ij')
    fr_, mk_, xyz = fisheye.pairwise_points(fr.ravel(), ca.ravel(), mk.ravel(), uv[..., 0].ravel(),
                                            uv[..., 1].ravel(), g['K'], g['D'], g['R'], g['t'])
    s0 = oekf.initial_state(mode, fr_, mk_, xyz, 0, 1 / 90.0)
    return g, s0


# EKF tolerances vs the reference run: the filter amplifies rounding-level differences
# (a 1e-13 relative change of s0 moves x by ~1e-8 two frames later, in float64 too), and
# the reference rounds its state to float32 each frame. head (40 frames): x 5e-5, dx 5e-4,
# ddx 5e-3 (|ddx| ~ 50), smoothed x 2e-5. default: the reference run itself diverges after
# frame ~18 (tail angles run away), so frames 0-9 only: x 1e-3.
EKF_TOL = {'x': 5e-5, 'dx': 5e-4, 'ddx': 5e-3, 'smoothed_x': 2e-5}


def test_oracle_ekf_matches_reference_head():
    from oracle import ekf as oekf
    g, s0 = _ekf_golden('head')
    out = oekf.ekf(g['uv'], g['likelihood'], g['K'], g['D'], g['R'], g['t'], 'head', 90.0, s0, 0.5,
                   float(g['res'][0]))
    P = 6
    xe, xs = out['x_est'], out['x_smooth']
    np.testing.assert_allclose(xe[:, :P], g['out_x'], atol=EKF_TOL['x'], rtol=0)
    np.testing.assert_allclose(xe[:, P:2 * P], g['out_dx'], atol=EKF_TOL['dx'], rtol=0)
    np.testing.assert_allclose(xe[:, 2 * P:], g['out_ddx'], atol=EKF_TOL['ddx'], rtol=0)
    np.testing.assert_allclose(xs[:, :P], g['out_smoothed_x'], atol=EKF_TOL['smoothed_x'], rtol=0)
    # first frame: same arithmetic up to float64 rounding
    np.testing.assert_allclose(xe[0, :P], g['out_x'][0], atol=1e-10, rtol=0)


def test_oracle_ekf_matches_reference_default_early_frames():
    from oracle import ekf as oekf
    g, s0 = _ekf_golden('default')
    out = oekf.ekf(g['uv'][:10], g['likelihood'][:10], g['K'], g['D'], g['R'], g['t'], 'default', 90.0, s0, 0.5,
                   float(g['res'][0]))
    np.testing.assert_allclose(out['x_est'][:, :29], g['out_x'][:10], atol=1e-3, rtol=0)
    np.testing.assert_allclose(out['x_est'][:2, :29], g['out_x'][:2], atol=1e-8, rtol=0)



@pytest.mark.parametrize('mode', ['head', 'default'])
def test_oracle_ekf_analytic_jacobian_matches_fd(mode):
    """The analytic H against central differences of the same float64
    measurement function, and the analytic-H filter tracking the reference's FD-H run on
    the head fixture (the two Jacobians differ by the FD truncation, O(eps))."""
    from oracle import ekf as oekf
    from acinoset_amd import synth
    sc = synth.load_scene_file()
    P = len(pkin.get_pose_params(mode))
    x = np.random.default_rng(5).normal(0, 0.1, P)
    x[:3] = [1.9, 6.4, 0.6]
    for c in range(sc.n_cams):
        h, H = oekf.analytic_jacobian(x, mode, sc.K[c], sc.D[c], sc.R[c], sc.t[c])
        Hc = np.empty_like(H)
        for i in range(P):
            d = np.zeros(P)
            d[i] = 1e-6
            hp = oekf.h_function(x + d, mode, sc.K[c], sc.D[c], sc.R[c], sc.t[c], ref_numerics=False).ravel()
            hm = oekf.h_function(x - d, mode, sc.K[c], sc.D[c], sc.R[c], sc.t[c], ref_numerics=False).ravel()
            Hc[:, i] = (hp - hm) / 2e-6
        np.testing.assert_allclose(h, oekf.h_function(x, mode, sc.K[c], sc.D[c], sc.R[c], sc.t[c],
                                                      ref_numerics=False).ravel(), rtol=0, atol=1e-9)
        np.testing.assert_allclose(H, Hc, rtol=0, atol=1e-6 * np.abs(H).max())
    if mode == 'head':
        g, s0 = _ekf_golden('head')
        out = oekf.ekf(g['uv'], g['likelihood'], g['K'], g['D'], g['R'], g['t'], 'head', 90.0, s0, 0.5,
                       float(g['res'][0]), ref_numerics=False, jacobian='analytic')
        assert np.sqrt(np.mean((out['x_smooth'][:, :6] - g['out_smoothed_x']) ** 2)) < 1e-2


# ---- FTE objective (parity unpinned vs IPOPT, oracle/fte.py): exact gradient and the
# shutter-delay modes (src/core/fte.py:236-238, :304-318, :447-450)
def _fte_small(sd_mode, inter, N=6, tau_max=0.004):
    from oracle import fte as ofte
    from acinoset_amd import synth
    scene = synth.load_scene_file()
    seq = synth.make_sequence(N, scene, mode='head', seed=2, tau_max=tau_max)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem('head', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True, intermode=inter,
                        sd_mode=sd_mode)
    return seq, prob


@pytest.mark.parametrize('sd_mode', ['const', 'variable'])
@pytest.mark.parametrize('inter', ['vel', 'acc'])
def test_oracle_fte_gradient_fd(sd_mode, inter):
    seq, prob = _fte_small(sd_mode, inter)
    rng = np.random.default_rng(1)
    X = np.concatenate([seq.x[:1], seq.x[:1], seq.x], 0) + rng.normal(0, 0.01, (prob.M, prob.P))
    tau = rng.uniform(-0.003, 0.003, prob.tau_shape)
    tau[..., 0] = 0.0
    F, H, g = prob.linearize(X, tau)
    assert F == prob.cost(X, tau)[0]
    v = prob.pack(X, tau)
    fd = np.zeros_like(v)
    for i in range(v.size):
        h = 1e-6 if i < prob.M * prob.P else 1e-8
        vp, vm = v.copy(), v.copy()
        vp[i] += h
        vm[i] -= h
        fd[i] = (prob.cost(*prob.unpack(vp))[0] - prob.cost(*prob.unpack(vm))[0]) / (2 * h)
    fd[prob.pinned()] = 0.0          # camera 0's delay is not an unknown
    np.testing.assert_allclose(g, fd, rtol=0, atol=1e-8 * np.abs(g).max())
    assert H.shape == (prob.nv, prob.nv)


def test_oracle_fte_variable_generalises_const():
    """tau[n, c] = tau_c for every n gives the const-mode objective; the variable optimum
    is at most the const one (a superset of the unknowns) and respects |tau| <= Ts."""
    from oracle import fte as ofte
    seq, pc = _fte_small('const', 'vel')
    _, pv = _fte_small('variable', 'vel')
    rng = np.random.default_rng(3)
    X = np.concatenate([seq.x[:1], seq.x[:1], seq.x], 0) + rng.normal(0, 0.01, (pc.M, pc.P))
    tc = np.array([0.0, 0.002, -0.001, 0.003, 0.0, -0.002])
    assert pv.cost(X, np.tile(tc, (pv.N, 1)))[0] == pytest.approx(pc.cost(X, tc)[0], rel=1e-14)
    X0 = ofte.initial_state(pc, np.arange(pc.N), seq.pos3d[:, 0, 0])
    _, tc_, ic = ofte.solve(pc, X0)
    _, tv_, iv = ofte.solve(pv, X0)
    assert iv['status'] in ('ftol', 'xtol', 'gtol') and ic['status'] in ('ftol', 'xtol', 'gtol')
    assert iv['cost_after'] <= ic['cost_after']
    assert np.all(np.abs(tv_) <= pv.Ts) and np.all(tv_[:, 0] == 0.0)


def test_oracle_fte_const_delay_at_bound():
    """A true delay beyond Ts drives tau_c to the bound; the active-set step keeps the
    solve converging there (held delays leave the gradient test)."""
    from oracle import fte as ofte
    seq, prob = _fte_small('const', 'vel', N=8, tau_max=0.03)
    X0 = ofte.initial_state(prob, np.arange(prob.N), seq.pos3d[:, 0, 0])
    _, tau, info = ofte.solve(prob, X0)
    assert info['status'] in ('ftol', 'xtol', 'gtol'), info
    assert np.any(np.abs(tau) == prob.Ts)
