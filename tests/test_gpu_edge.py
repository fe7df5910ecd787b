"""GPU edge cases at the size limits of the kernels, against the oracle:

* SBA observation lists with many observations per point (slot groups of 64 lanes, and
  more slots than lanes: K = 100 and the maximum K = 256 take the 4-slots-per-lane kernel),
  ragged counts;
* FTE at the smallest trajectories (N = 2, 3, 4 frames: one or two super-blocks, zero or
  one cyclic-reduction level) and with two cameras; max_iters = 0; frames without a single
  observation (zero weights);
* EKF frames whose likelihoods are all below the threshold (prediction only).

Tolerances as the main parity tests: SBA points 1e-7 m; FTE keypoints 1e-6 m RMS, tau
1e-6 s, same accept count.
"""
import numpy as np
import pytest

from acinoset_amd import _native, kinematics as pkin, synth
from oracle import fisheye, fte as ofte, kinematics as okin, sba as osba

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('kmax', [40, 100, 256])
def test_sba_many_observations_per_point(ctx, kmax):
    scene = synth.load_scene_file()
    C = scene.n_cams
    rng = np.random.default_rng(kmax)
    n = 96
    X = np.array([1.9, 6.4, 0.5]) + rng.normal(0, 0.3, (n, 3))
    counts = rng.integers(2, kmax + 1, n)                 # ragged: 2 .. kmax observations
    counts[0] = kmax
    pi = np.repeat(np.arange(n), counts).astype(np.int32)
    ci = rng.integers(0, C, len(pi)).astype(np.int32)
    uv = fisheye.project(X[pi], scene.K[ci], scene.D[ci], scene.R[ci], scene.t[ci])
    uv = uv + rng.normal(0, 1.0, uv.shape)
    uv[rng.random(len(uv)) < 0.02] += 40.0                # a few outliers
    perm = rng.permutation(len(pi))                       # arbitrary observation order
    pi, ci, uv = pi[perm], ci[perm], uv[perm]
    X0 = X + rng.normal(0, 0.02, X.shape)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    pts, rb, ra, rep = ctx.sba_points(cams, uv, pi, ci, X0)
    ref = osba.sba_points(uv, X0, pi, ci, scene.K, scene.D, scene.R, scene.t)
    assert float(np.abs(pts - ref).max()) < 1e-7
    st = rep['status_counts']
    assert st['running'] == st['stalled'] == st['maxiter'] == 0, st


def _fte_problem(N, cams=None, seed=5):
    scene = synth.load_scene_file()
    if cams is not None:
        scene = scene.subset(cams)
    seq = synth.make_sequence(N, scene, mode='default_nolure', seed=seed, tau_max=0.004)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                        intermode='vel')
    X0 = np.concatenate([seq.x[:1], seq.x[:1], seq.x], 0) + np.random.default_rng(seed).normal(0, 0.01, (N + 2, prob.P))
    return seq, prob, _native.pack_cameras(scene.K, scene.D, scene.R, scene.t), X0


@pytest.mark.parametrize('N,cams', [(2, None), (3, None), (4, None), (25, [0, 3])])
def test_fte_smallest_trajectories_match_oracle(ctx, N, cams):
    seq, prob, pc, X0 = _fte_problem(N, cams)
    table = pkin.build_table(prob.mode)
    X, tau, rep = ctx.fte_solve(table, pc, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=60))
    Xo, to, info = ofte.solve(prob, X0, max_iters=60)
    assert rep['n_accepted'] == info['n_accepted'], (rep, info)
    pg = okin.marker_positions(prob.mode, X[2:])
    po = okin.marker_positions(prob.mode, Xo[2:])
    assert float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1)))) < 1e-6
    np.testing.assert_allclose(tau, to, rtol=0, atol=1e-6)


def _fte20():
    scene = synth.load_scene_file()
    seq = synth.make_sequence(20, scene, mode='default_nolure', seed=2, tau_max=0.004)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    return scene, seq, w, cams


def test_fte_max_iters_zero_returns_start(ctx):
    scene, seq, w, cams = _fte20()
    prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                        intermode='vel')
    X0 = ofte.initial_state(prob, np.arange(20), seq.pos3d[:, 0, 0])
    X, tau, rep = ctx.fte_solve(pkin.build_table('default_nolure'), cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=0))
    Xo, to, info = ofte.solve(prob, X0, max_iters=0)
    assert rep['status_name'] == info['status'] == 'maxiter' and rep['iters'] == info['iters'] == 0
    np.testing.assert_array_equal(X, X0)
    assert abs(rep['cost_after'] - info['cost_after']) <= 1e-12 * info['cost_after']


def test_fte_frames_without_observations_match_oracle(ctx):
    """Two consecutive frames with every weight zero: only the motion model holds them."""
    scene, seq, w, cams = _fte20()
    w[5:7] = 0.0
    prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                        intermode='vel')
    X0 = ofte.initial_state(prob, np.arange(20), seq.pos3d[:, 0, 0])
    X, tau, rep = ctx.fte_solve(pkin.build_table('default_nolure'), cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    Xo, to, info = ofte.solve(prob, X0)
    assert rep['status_name'] == info['status'] and rep['iters'] == info['iters'], (rep, info)
    pg = okin.marker_positions(prob.mode, X[2:])
    po = okin.marker_positions(prob.mode, Xo[2:])
    assert float(np.sqrt(np.mean(np.sum((pg - po) ** 2, -1)))) < 1e-6
    np.testing.assert_allclose(tau, to, rtol=0, atol=1e-6)
    assert abs(rep['cost_after'] - info['cost_after']) <= 1e-9 * info['cost_after']


def test_ekf_frames_below_threshold_match_oracle(ctx):
    """Frames 3-5 with every likelihood below the threshold (no update, prediction only), head
    model, 12-camera ring, float64: the 12-camera tolerances of tests/test_gpu_ekf.py."""
    import importlib
    from oracle import ekf as oekf
    from test_gpu_ekf import TOL, _setup_ring
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    scene, seq, s0, cp, covs = _setup_ring('head', 12)
    lik = seq.likelihood.copy()
    lik[3:6] = 0.0
    out = cekf.run(seq.uv, lik, cp, 'head', 90.0, s0, ref_numerics=False, cal_covs=covs, ctx=ctx)
    o = oekf.ekf(seq.uv, lik, scene.K, scene.D, scene.R, scene.t, 'head', 90.0, s0, 0.5, float(scene.res[0]),
                 ref_numerics=False, cal_covs=covs)
    P = 6
    np.testing.assert_allclose(out['x_est'][:, :P], o['x_est'][:, :P], rtol=0, atol=TOL['x'])
    np.testing.assert_allclose(out['x_est'][:, P:2 * P], o['x_est'][:, P:2 * P], rtol=0, atol=TOL['dx'])
    np.testing.assert_allclose(out['x_est'][:, 2 * P:], o['x_est'][:, 2 * P:], rtol=0, atol=TOL['ddx'])
    np.testing.assert_allclose(out['x_smooth'][:, :P], o['x_smooth'][:, :P], rtol=0, atol=TOL['smoothed_x'])
    assert int(out['outliers']) == o['outliers']

