"""GPU parity: bundle adjustment of points AND extrinsics (acs_sba_extrinsics, §8(a) a6)
against oracle/sba_ext.py (same Schur-complement LM spec) and the reference's golden run
of bundle_adjust_points_and_extrinsics (src/lib/sba.py:158-178).

Tolerances (float64 both sides): the oracle and the kernels run the same LM iteration by
iteration, but sum the reduced camera system in different orders, so the iterates agree
to rounding (the damping floor 1e-7 keeps the free 7-DoF gauge from amplifying it):
iteration counts exact, cost rel 1e-12, points/translations 1e-9 m, rotations 1e-10,
residuals 1e-8 px. Against the reference: cost no larger than scipy's final cost."""
import numpy as np
import pytest

from conftest import golden
from oracle import sba_ext as oext
from acinoset_amd import _native

pytestmark = pytest.mark.gpu


def _problem(g):
    return (_native.pack_cameras(g['K'], g['D'], g['R0'], g['t0']), g['points_2d'], g['point_indices'],
            g['camera_indices'], g['points_3d'])


def _oracle(g, **kw):
    return oext.sba_extrinsics(g['points_2d'], g['points_3d'], g['point_indices'].astype(np.int64),
                               g['camera_indices'].astype(np.int64), g['K'], g['D'].reshape(-1, 4), g['R0'], g['t0'],
                               **kw)


@pytest.mark.parametrize('max_iters', [1, 5, 20, 200])
def test_sba_ext_matches_oracle(ctx, max_iters):
    g = golden('sba_extrinsics')
    cams, uv, pi, ci, X0 = _problem(g)
    o = ctx.sba_ext_opts(max_iters=max_iters)
    cams_out, X, rb, ra, rep = ctx.sba_extrinsics(cams, uv, pi, ci, X0, o)
    Xo, Ro, to, info = _oracle(g, max_iters=max_iters)
    np.testing.assert_allclose(rb, g['resid_before'], atol=1e-9)
    assert rep['status_name'] == info['status']
    # the same accept/reject sequence, iterate for iterate
    assert rep['iters'] == info['iters'] and rep['n_accepted'] == info['n_accepted']
    assert abs(rep['lambda_final'] - info['lam']) <= 1e-12 * info['lam']
    assert abs(rep['cost_before'] - info['cost_before']) <= 1e-12 * info['cost_before']
    assert abs(rep['cost_after'] - info['cost_after']) <= 1e-12 * info['cost_after']
    np.testing.assert_allclose(X, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(cams_out[:, 8:17].reshape(-1, 3, 3), Ro, rtol=0, atol=1e-10)
    np.testing.assert_allclose(cams_out[:, 17:20], to.reshape(-1, 3), rtol=0, atol=1e-9)
    ro = oext.residuals(Xo, Ro, to, g['K'], g['D'].reshape(-1, 4), uv, pi, ci).ravel()
    np.testing.assert_allclose(ra, ro, atol=1e-8)
    R = cams_out[:, 8:17].reshape(-1, 3, 3)
    np.testing.assert_allclose(R @ np.swapaxes(R, 1, 2), np.broadcast_to(np.eye(3), R.shape), atol=1e-12)
    np.testing.assert_array_equal(cams_out[:, :8], cams[:, :8])  # intrinsics untouched


def test_sba_ext_beats_reference(ctx):
    from acinoset_amd.lib import sba as lsba
    g = golden('sba_extrinsics')
    obj, R, t, res = lsba.bundle_adjust_points_and_extrinsics(g['points_2d'], g['points_3d'], g['point_indices'],
                                                              g['camera_indices'], g['K'], g['D'], g['R0'], g['t0'],
                                                              None)
    assert obj.shape == (80, 3) and R.shape == (6, 3, 3) and t.shape == (6, 3, 1)
    np.testing.assert_allclose(res['before'], g['resid_before'], atol=1e-9)
    c_ref = 0.5 * np.log1p(g['resid_after'] ** 2).sum()
    c_ours = 0.5 * np.log1p(res['after'] ** 2).sum()
    assert c_ours <= c_ref
    # the returned state reproduces the returned residuals
    r = oext.residuals(obj, R, t.reshape(-1, 3), g['K'], g['D'].reshape(-1, 4), g['points_2d'], g['point_indices'],
                       g['camera_indices']).ravel()
    np.testing.assert_allclose(r, res['after'], atol=1e-9)


def _synthetic(n_pts, C, seed, perturb=True):
    from acinoset_amd import synth
    rng = np.random.default_rng(seed)
    sc = synth.ring_scene(C)
    K, D, R, t = sc.K, sc.D, sc.R, sc.t
    X = rng.uniform(-2, 2, (n_pts, 3)) * [1, 1, 0.3] + [1.9, 6.4, 0.5]
    pi, ci = [], []
    for p in range(n_pts):
        cs = rng.choice(C, size=rng.integers(2, C + 1), replace=False)
        pi += [p] * len(cs)
        ci += list(cs)
    pi, ci = np.array(pi, np.int32), np.array(ci, np.int32)
    uv = oext.residuals(X, R, t.reshape(-1, 3), K, D.reshape(-1, 4), np.zeros((len(pi), 2)), pi, ci)
    R0, t0, X0 = R.copy(), t.copy().reshape(-1, 3), X.copy()
    if perturb:
        for c in range(1, C):
            R0[c] = oext.rodrigues(rng.normal(0, 2e-3, 3)) @ R0[c]
            t0[c] += rng.normal(0, 5e-3, 3)
        X0 = X + rng.normal(0, 5e-3, X.shape)
    return K, D, R0, t0, X0, uv, pi, ci


def test_sba_ext_synthetic_noiseless_converges(ctx):
    K, D, R0, t0, X0, uv, pi, ci = _synthetic(600, 8, 3)
    cams = _native.pack_cameras(K, D, R0, t0)
    o = ctx.sba_ext_opts(max_iters=300, f_scale=5.0)
    _, X, rb, ra, rep = ctx.sba_extrinsics(cams, uv, pi, ci, X0, o)
    assert np.sqrt(np.mean(ra ** 2)) < 1e-6 < np.sqrt(np.mean(rb ** 2))
    assert rep['n_bad_pivots'] == 0


@pytest.mark.parametrize('C', [12, 16])
def test_sba_ext_many_cameras_matches_oracle(ctx, C):
    """A ring of 12 / 16 cameras (EXT_MAXC = 16: a 96 x 96 reduced camera system), 0.5 px
    noise, 20 iterations, against the oracle at test_sba_ext_matches_oracle's tolerances."""
    K, D, R0, t0, X0, uv, pi, ci = _synthetic(400, C, 11)
    uv = uv + np.random.default_rng(12).normal(0, 0.5, uv.shape)
    cams = _native.pack_cameras(K, D, R0, t0)
    cams_out, X, rb, ra, rep = ctx.sba_extrinsics(cams, uv, pi, ci, X0, ctx.sba_ext_opts(max_iters=20))
    Xo, Ro, to, info = oext.sba_extrinsics(uv, X0, pi.astype(np.int64), ci.astype(np.int64), K, D.reshape(-1, 4),
                                           R0, t0, max_iters=20)
    assert rep['status_name'] == info['status'] and rep['n_bad_pivots'] == 0
    assert rep['iters'] == info['iters'] and rep['n_accepted'] == info['n_accepted']
    assert abs(rep['cost_after'] - info['cost_after']) <= 1e-12 * info['cost_after']
    np.testing.assert_allclose(X, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(cams_out[:, 8:17].reshape(-1, 3, 3), Ro, rtol=0, atol=1e-10)
    np.testing.assert_allclose(cams_out[:, 17:20], to.reshape(-1, 3), rtol=0, atol=1e-9)


def test_sba_ext_unobserved_point_and_order_invariance(ctx):
    K, D, R0, t0, X0, uv, pi, ci = _synthetic(100, 6, 5)
    X0 = np.vstack([X0, [[0.1, 0.2, 0.3]]])  # point 100 has no observations
    cams = _native.pack_cameras(K, D, R0, t0)
    o = ctx.sba_ext_opts(max_iters=20)
    c1, X1, _, ra1, rep1 = ctx.sba_extrinsics(cams, uv, pi, ci, X0, o)
    assert np.all(np.isfinite(X1)) and np.array_equal(X1[100], X0[100])
    perm = np.random.default_rng(1).permutation(len(pi))
    c2, X2, _, ra2, rep2 = ctx.sba_extrinsics(cams, uv[perm], pi[perm], ci[perm], X0, o)
    # observations are regrouped per point; a permutation changes only the slot order
    # within a point, i.e. the summation order of its few terms
    assert rep1['iters'] == rep2['iters']
    np.testing.assert_allclose(X1, X2, rtol=0, atol=1e-9)
    np.testing.assert_allclose(c1, c2, rtol=0, atol=1e-9)


def test_sba_ext_bad_inputs(ctx):
    g = golden('sba_extrinsics')
    cams, uv, pi, ci, X0 = _problem(g)
    with pytest.raises(RuntimeError):
        ctx.sba_extrinsics(np.tile(cams, (3, 1)), uv, pi, ci, X0)  # 18 cameras > 16
    bad = pi.copy()
    bad[0] = 10_000
    with pytest.raises(RuntimeError):
        ctx.sba_extrinsics(cams, uv, bad, ci, X0)
