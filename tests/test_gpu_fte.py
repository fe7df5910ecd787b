"""GPU parity of the FTE trajectory solve (acs_fte_eval / acs_fte_solve) against the
oracle restatement of src/core/fte.py (parity unpinned vs IPOPT: see oracle/fte.py),
both shutter-delay modes (const: tau (C,), variable: tau (N, C), src/core/fte.py:236-238).

Tolerances (float64):
  * objective: 1e-10 relative; gradient / GN normal matrix: 1e-8 relative to their max
  * solution vs oracle (same LM spec): 1e-6 m RMS keypoint position (contract 1e-4 m),
    reprojection RMS within 1e-3 px (north_star), tau within 1e-6 s
  * one LM step (the cyclic-reduction solve of the damped normal equations): 1e-9
"""
import numpy as np
import pytest

from oracle import fte as ofte, kinematics as okin
from acinoset_amd import _native, kinematics as pkin, synth

pytestmark = pytest.mark.gpu


def _problem(N, mode='default_nolure', sd=True, inter='vel', seed=2, tau_max=0.004, sd_mode='const', n_cams=None):
    scene = synth.load_scene_file() if n_cams is None else synth.ring_scene(n_cams)
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed, tau_max=tau_max if sd else 0.0)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem(mode, seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=sd, intermode=inter,
                        sd_mode=sd_mode)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    return seq, prob, cams


def _reproj_rms(prob, X, tau):
    e = prob.residuals(X, tau) * 3.0            # back to pixels (w = 1/3)
    m = prob.w > 0
    return float(np.sqrt(np.mean(np.sum(e[m] ** 2, -1))))


@pytest.mark.parametrize('sd,inter', [(False, 'pos'), (True, 'vel'), (True, 'acc')])
def test_fte_eval_matches_oracle(ctx, sd, inter):
    seq, prob, cams = _problem(12, sd=sd, inter=inter)
    rng = np.random.default_rng(4)
    X = np.concatenate([seq.x[:1], seq.x[:1], seq.x], 0) + rng.normal(0, 0.01, (prob.M, prob.P))
    tau = np.array([0.0, 0.002, -0.001, 0.003, 0.0, -0.002]) if sd else np.zeros(6)
    table = pkin.build_table(prob.mode)
    cost, g, H = ctx.fte_eval(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X, tau, shutter_delay=sd,
                              intermode=prob.im)
    F = prob.cost(X, tau)
    np.testing.assert_allclose(cost, F, rtol=1e-10)
    Fo, Ho, go = prob.linearize(X, tau)
    go = go.copy()
    if sd:
        go[prob.M * prob.P] = 0.0
    np.testing.assert_allclose(g, go, rtol=0, atol=1e-8 * np.abs(go).max())
    Hd = Ho.toarray()
    np.testing.assert_allclose(H, Hd, rtol=0, atol=1e-8 * np.abs(Hd).max())


@pytest.mark.parametrize('mode,sd,inter,N', [('default_nolure', True, 'vel', 40), ('head', True, 'vel', 60),
                                             ('upper_body', True, 'vel', 30),
                                             ('default_nolure', False, 'pos', 30),
                                             ('default_nolure', True, 'acc', 30)])
def test_fte_solve_matches_oracle(ctx, mode, sd, inter, N):
    seq, prob, cams = _problem(N, mode=mode, sd=sd, inter=inter)
    nose = seq.pos3d[:, 0, 0]
    X0 = ofte.initial_state(prob, np.arange(N), nose)
    Xo, to, info = ofte.solve(prob, X0)
    table = pkin.build_table(mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, shutter_delay=sd,
                                intermode=prob.im)
    assert rep['status_name'] in ('ftol', 'xtol', 'gtol'), rep
    assert info['status'] in ('ftol', 'xtol', 'gtol'), info
    pg = okin.marker_positions(mode, X[2:])
    po = okin.marker_positions(mode, Xo[2:])
    rms = float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1))))
    assert rms < 1e-6, (rms, rep, info)
    assert abs(_reproj_rms(prob, X, tau) - _reproj_rms(prob, Xo, to)) < 1e-3
    np.testing.assert_allclose(tau, to, atol=1e-6)
    np.testing.assert_allclose(rep['cost_after'], info['cost_after'], rtol=1e-9, atol=1e-9)
    # and the solve actually fits the data: keypoints within a few mm of the truth
    truth = seq.pos3d[:, 0]
    assert float(np.sqrt(np.mean(np.sum((pg - truth) ** 2, -1)))) < 0.02


@pytest.mark.parametrize('N', [7, 31, 64])
def test_fte_single_lm_step_matches_oracle(ctx, N):
    """One LM step (lambda0) = one solve of the damped normal equations: checks the
    block-cyclic-reduction linear solve (odd/even/power-of-two super-block counts)."""
    seq, prob, cams = _problem(N)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=1))
    Xo, to, info = ofte.solve(prob, X0, max_iters=1)
    assert rep['n_bad_pivots'] == 0 and rep['iters'] == 1 and info['iters'] == 1
    assert rep['n_accepted'] == info['n_accepted']
    np.testing.assert_allclose(X, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(tau, to, rtol=0, atol=1e-12)


def test_fte_deterministic(ctx):
    seq, prob, cams = _problem(30)
    X0 = ofte.initial_state(prob, np.arange(30), seq.pos3d[:, 0, 0])
    table = pkin.build_table(prob.mode)
    a = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    b = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_fte_rejects_bad_modes(ctx):
    seq, prob, cams = _problem(8)
    table = pkin.build_table(prob.mode)
    X0 = np.zeros((prob.M, prob.P))
    with pytest.raises(RuntimeError):   # shutter delay with intermode 'pos' (fte.py:44-46)
        ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, shutter_delay=True, intermode=0)


# ---- shutter_delay_mode='variable' (per-frame delays eliminated frame by frame) ---------
@pytest.mark.parametrize('inter', ['vel', 'acc'])
def test_fte_eval_variable_matches_oracle(ctx, inter):
    seq, prob, cams = _problem(10, sd_mode='variable', inter=inter)
    rng = np.random.default_rng(5)
    X = np.concatenate([seq.x[:1], seq.x[:1], seq.x], 0) + rng.normal(0, 0.01, (prob.M, prob.P))
    tau = rng.uniform(-0.004, 0.004, (prob.N, prob.C))
    tau[:, 0] = 0.0
    table = pkin.build_table(prob.mode)
    cost, g, H = ctx.fte_eval(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X, tau, intermode=prob.im,
                              sd_mode='variable')
    np.testing.assert_allclose(cost, prob.cost(X, tau), rtol=1e-10)
    Fo, Ho, go = prob.linearize(X, tau)
    np.testing.assert_allclose(g, go, rtol=0, atol=1e-8 * np.abs(go).max())
    Hd = Ho.toarray()
    np.testing.assert_allclose(H, Hd, rtol=0, atol=1e-8 * np.abs(Hd).max())


@pytest.mark.parametrize('N,iters', [(7, 1), (31, 1), (64, 1), (31, 5)])
def test_fte_variable_lm_steps_match_oracle(ctx, N, iters):
    """The first LM steps: per-frame delay elimination + cyclic reduction + delay
    back-substitution = the oracle's sparse solve of the full damped system."""
    seq, prob, cams = _problem(N, sd_mode='variable')
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=iters), sd_mode='variable')
    Xo, to, info = ofte.solve(prob, X0, max_iters=iters)
    assert tau.shape == (N, prob.C)
    assert rep['n_bad_pivots'] == 0 and rep['iters'] == info['iters'] and rep['n_accepted'] == info['n_accepted']
    np.testing.assert_allclose(X, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(tau, to, rtol=0, atol=1e-11)


@pytest.mark.parametrize('mode,inter,N', [('default_nolure', 'vel', 30), ('head', 'acc', 40)])
def test_fte_variable_solve_matches_oracle(ctx, mode, inter, N):
    seq, prob, cams = _problem(N, mode=mode, inter=inter, sd_mode='variable')
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    Xo, to, info = ofte.solve(prob, X0)
    table = pkin.build_table(mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, intermode=prob.im,
                                sd_mode='variable')
    assert rep['status_name'] in ('ftol', 'xtol', 'gtol'), rep
    assert info['status'] in ('ftol', 'xtol', 'gtol'), info
    pg = okin.marker_positions(mode, X[2:])
    po = okin.marker_positions(mode, Xo[2:])
    assert float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1)))) < 1e-6
    np.testing.assert_allclose(tau, to, atol=1e-6)
    np.testing.assert_allclose(rep['cost_after'], info['cost_after'], rtol=1e-9, atol=1e-9)
    assert np.all(np.abs(tau) <= prob.Ts) and np.all(tau[:, 0] == 0.0)


def test_fte_const_delay_at_bound_matches_oracle(ctx):
    """True delays beyond Ts: the const-mode delays end on the bound (active set)."""
    seq, prob, cams = _problem(30, tau_max=0.03)
    X0 = ofte.initial_state(prob, np.arange(30), seq.pos3d[:, 0, 0])
    Xo, to, info = ofte.solve(prob, X0)
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    assert np.any(np.abs(to) == prob.Ts)
    assert rep['iters'] == info['iters'] and rep['status_name'] == info['status'], (rep, info)
    np.testing.assert_allclose(X, Xo, rtol=0, atol=1e-6)
    np.testing.assert_allclose(tau, to, rtol=0, atol=1e-9)


@pytest.mark.parametrize('sd_mode', ['const', 'variable'])
def test_fte_rejected_steps_match_oracle(ctx, sd_mode):
    """A start 1.5 rad off in every joint angle forces rejected LM steps. This covers the
    speculative double-buffered linearisation: a rejected trial overwriting the spare
    buffer, the next iteration re-assembling from the kept one (and, with variable delays,
    re-eliminating the per-frame delays), and a later accept flipping the buffers."""
    N = 40
    seq, prob, cams = _problem(N, sd_mode=sd_mode)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0]).copy()
    X0[:, 3:] += 1.5
    Xo, to, info = ofte.solve(prob, X0, max_iters=40)
    assert info['n_accepted'] < info['iters']
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=40), sd_mode=sd_mode)
    assert rep['iters'] == info['iters'] and rep['n_accepted'] == info['n_accepted'], (rep, info)
    assert rep['status_name'] == info['status'], (rep, info)
    # same accept/reject sequence (above); the iterates themselves are mid-path (max_iters,
    # lambda at its floor, far from the optimum), where 40 iterations amplify the
    # summation-order differences (1e-12 after the first step) to ~1e-5 m: compared at the
    # north_star contract (1e-4 m RMS), cost to 1e-6 relative, tau to 5e-5 s (the
    # per-frame delays of the variable mode are weakly determined mid-path; Ts = 0.011 s)
    pg = okin.marker_positions(prob.mode, X[2:])
    po = okin.marker_positions(prob.mode, Xo[2:])
    assert float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1)))) < 1e-4
    np.testing.assert_allclose(tau, to, rtol=0, atol=5e-5)
    np.testing.assert_allclose(rep['cost_after'], info['cost_after'], rtol=1e-6)


@pytest.mark.parametrize('n_cams,mode,sd_mode', [(12, 'default_nolure', 'const'), (16, 'default_nolure', 'const'),
                                                (12, 'default_nolure', 'variable'), (16, 'default', 'const'),
                                                (16, 'head', 'const'), (16, 'upper_body', 'const')])
def test_fte_many_cameras_matches_oracle(ctx, n_cams, mode, sd_mode):
    """More observations per frame than one aggregation chunk of k_fte_linearize (LIN_OCH =
    128; 12 and 16 cameras x 20-21 markers = 240-336), so the observation sums run over 2-3
    chunks. A constant shutter delay per camera gives a tau border of 12 or 16 delays: at 16
    (FTE_MAXC) the border plus the gradient column is two column-blocks (GR = 32) and
    k_cr_level reads E_r from global memory (cr_er_lds). 'default' (with the lure, P = 29)
    takes the 96-row super-blocks (NB = 6); 'head' and 'upper_body' (3 and 7 markers: one
    chunk) the 32- and 48-row ones (NB = 2, 3), whose deep levels deal one column-block per
    workgroup. A ring of cameras (synth.ring_scene), solved to convergence, against the
    oracle at the contract of test_fte_solve_matches_oracle."""
    N = 20
    seq, prob, cams = _problem(N, mode=mode, n_cams=n_cams, sd_mode=sd_mode)
    assert seq.uv.shape[1] == n_cams and (mode in ('head', 'upper_body') or n_cams * seq.uv.shape[2] > 128)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    Xo, to, info = ofte.solve(prob, X0)
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, sd_mode=sd_mode)
    assert rep['status_name'] in ('ftol', 'xtol', 'gtol'), rep
    assert info['status'] in ('ftol', 'xtol', 'gtol'), info
    assert rep['iters'] == info['iters'], (rep, info)
    pg = okin.marker_positions(prob.mode, X[2:])
    po = okin.marker_positions(prob.mode, Xo[2:])
    rms = float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1))))
    assert rms < 1e-6, (rms, rep, info)
    assert abs(_reproj_rms(prob, X, tau) - _reproj_rms(prob, Xo, to)) < 1e-3
    np.testing.assert_allclose(tau, to, atol=1e-6)
    np.testing.assert_allclose(rep['cost_after'], info['cost_after'], rtol=1e-9, atol=1e-9)
    # the fit itself (the oracle's too): within a few cm of the truth (the 3-marker head model
    # with 16 free delays: 2.6 cm)
    truth = seq.pos3d[:, 0]
    assert float(np.sqrt(np.mean(np.sum((pg - truth) ** 2, -1)))) < 0.05
