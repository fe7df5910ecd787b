"""configs[4]: the fused SBA + EKF pipeline (acs_sba_ekf_pipeline) against the oracle pieces
run one after the other on the same observations:
  oracle/fisheye.pairwise_points (src/lib/utils.py:319-349) -> oracle/sba.sba_points on the
  observations of the triangulated points (src/lib/sba.py:285-313) -> oracle/ekf.initial_state
  (src/core/ekf.py:121-157) on the SBA (or triangulated) points -> oracle/ekf.ekf (:26-298).

Tolerances: SBA points 1e-7 m (as test_gpu_core's SBA parity), the NaN pattern (points no
adjacent pair saw) identical; the first filtered state 1e-9 (head) / 1e-7 (the 87-state
default model, whose initial state is fitted on SBA points that agree to ~4e-9 m); the EKF
states at the
test_gpu_ekf tolerances (x 5e-5, dx 5e-4, ddx 5e-3, smoothed x 2e-5; x10 for the 29-state
default model); outlier counts within 1 per sequence.
"""
import importlib

import numpy as np
import pytest

from oracle import ekf as oekf, fisheye as ofi, sba as osba
from acinoset_amd import _native, kinematics as pkin, synth

pytestmark = pytest.mark.gpu
cekf = importlib.import_module('acinoset_amd.core.ekf')
TOL = {'x': 5e-5, 'dx': 5e-4, 'ddx': 5e-3, 'smoothed_x': 2e-5}


def _oracle(scene, uv, lik, obs_markers, ekf_mode, thresh, from_sba, ref_numerics, covs, fps=90.0):
    """One sequence through the oracle pieces. Returns (pts (N, Lo, 3), s0, ekf dict)."""
    N, C, Lo, _ = uv.shape
    valid = (lik > thresh) & np.isfinite(uv).all(-1)
    f, c, l = np.nonzero(valid)
    fr, mk, xyz = ofi.pairwise_points(f, c, l, uv[f, c, l, 0], uv[f, c, l, 1], scene.K, scene.D, scene.R, scene.t)
    pid = {(a, b): i for i, (a, b) in enumerate(zip(fr, mk))}
    keep = np.array([(a, b) in pid for a, b in zip(f, l)], bool)
    pi = np.array([pid[(a, b)] for a, b in zip(f[keep], l[keep])], np.int64)
    pts_o = osba.sba_points(uv[f[keep], c[keep], l[keep]], xyz, pi, c[keep], scene.K, scene.D, scene.R, scene.t)
    pts = np.full((N, Lo, 3), np.nan)
    pts[fr, mk] = pts_o
    ekf_markers = pkin.get_markers(ekf_mode)
    to_e = np.array([ekf_markers.index(m) if m in ekf_markers else -1 for m in obs_markers])
    sel = to_e[mk] >= 0
    src = pts_o if from_sba else xyz
    s0 = oekf.initial_state(ekf_mode, fr[sel], to_e[mk[sel]], src[sel], 0, 1.0 / fps)
    cols = [obs_markers.index(m) for m in ekf_markers]
    o = oekf.ekf(uv[:, :, cols], lik[:, :, cols], scene.K, scene.D, scene.R, scene.t, ekf_mode, fps, s0, thresh,
                 float(scene.res[0]), ref_numerics=ref_numerics, cal_covs=covs)
    return pts, s0, o


def _run(ctx, n_cams, obs_mode, ekf_mode, n_seq, N, from_sba, ref_numerics, seed=71):
    scene = synth.load_scene_file() if n_cams == 6 else synth.ring_scene(n_cams)
    seqs = [synth.make_sequence(N, scene, mode=obs_mode, seed=seed + k) for k in range(n_seq)]
    uv = np.stack([q.uv for q in seqs])
    lik = np.stack([q.likelihood for q in seqs])
    table = pkin.build_table(ekf_mode)
    covs = cekf.ring_cal_covs(n_cams)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    P = table.P
    out = ctx.sba_ekf_pipeline(table, cams, uv, lik, seqs[0].markers, 90.0, 0.5, float(scene.res[0]),
                               cekf.measurement_std(n_cams, covs), cekf.process_covariance(P, 1 / 90.0),
                               cekf.initial_covariance(ekf_mode), from_sba=from_sba, ref_numerics=ref_numerics)
    return scene, seqs, uv, lik, covs, table, out


@pytest.mark.parametrize('from_sba,ref_numerics', [(True, False), (False, True)])
def test_pipeline_12cam_head_matches_oracle(ctx, from_sba, ref_numerics):
    """12-camera ring, 20-keypoint observations, the head EKF model on its 3 markers."""
    scene, seqs, uv, lik, covs, table, out = _run(ctx, 12, 'default_nolure', 'head', 2, 30, from_sba, ref_numerics)
    P = table.P
    assert out['sba']['n_problems'] == 2 * 30 * 20
    for k in range(len(seqs)):
        pts, s0, o = _oracle(scene, uv[k], lik[k], seqs[k].markers, 'head', 0.5, from_sba, ref_numerics, covs)
        g = out['pts'][k]
        np.testing.assert_array_equal(np.isnan(g), np.isnan(pts))
        m = ~np.isnan(pts)
        np.testing.assert_allclose(g[m], pts[m], rtol=0, atol=1e-7)
        xe, xs = out['x_est'][k], out['x_smooth'][k]
        # the filter's first state is s0 after one prediction + update: compare through it
        np.testing.assert_allclose(xe[0], o['x_est'][0], rtol=0, atol=1e-9)
        np.testing.assert_allclose(xe[:, :P], o['x_est'][:, :P], rtol=0, atol=TOL['x'])
        np.testing.assert_allclose(xe[:, P:2 * P], o['x_est'][:, P:2 * P], rtol=0, atol=TOL['dx'])
        np.testing.assert_allclose(xe[:, 2 * P:], o['x_est'][:, 2 * P:], rtol=0, atol=TOL['ddx'])
        np.testing.assert_allclose(xs[:, :P], o['x_smooth'][:, :P], rtol=0, atol=TOL['smoothed_x'])
        assert abs(int(out['outliers'][k]) - o['outliers']) <= 1
        # and the head is tracked
        pe = ctx.fk(table, np.ascontiguousarray(xs[:, :P]))
        assert float(np.sqrt(np.mean(np.sum((pe - seqs[k].pos3d[:, 0, :3]) ** 2, -1)))) < 0.05


@pytest.mark.parametrize('n_cams', [24, 40, 64])
def test_pipeline_many_cameras_matches_oracle(ctx, n_cams):
    """24-, 40- and 64-camera rings (64: the ABI maximum; SBA lane groups of 32 / 64 lanes; the EKF's per-frame observations grow with the cameras), head model on the SBA
    points, float64: SBA points 1e-7 m with the same NaN pattern, the EKF's marker positions
    within 1e-6 m of the oracle's (the state tolerances of the 12-camera test would flag the
    acceleration states, whose rounding-level differences grow with the measurement rows:
    profiles/r05/ekf_manycam_r05.log), outliers within 1."""
    from oracle import kinematics as okin
    scene, seqs, uv, lik, covs, table, out = _run(ctx, n_cams, 'default_nolure', 'head', 1, 20, True, False)
    P = table.P
    pts, s0, o = _oracle(scene, uv[0], lik[0], seqs[0].markers, 'head', 0.5, True, False, covs)
    g = out['pts'][0]
    np.testing.assert_array_equal(np.isnan(g), np.isnan(pts))
    m = ~np.isnan(pts)
    np.testing.assert_allclose(g[m], pts[m], rtol=0, atol=1e-7)
    for key in ('x_est', 'x_smooth'):
        d = np.abs(okin.marker_positions('head', out[key][0][:, :P]) - okin.marker_positions('head', o[key][:, :P]))
        assert d.max() < 1e-6, (key, d.max())
    assert abs(int(out['outliers'][0]) - o['outliers']) <= 1


def test_pipeline_6cam_default_model_matches_oracle(ctx):
    """The reference's 6-camera scene and its 21-marker 'default' model (identity marker
    map, lure line fit) over the frames before that filter loses the synthetic subject."""
    scene, seqs, uv, lik, covs, table, out = _run(ctx, 6, 'default', 'default', 1, 8, True, False, seed=81)
    P = table.P
    pts, s0, o = _oracle(scene, uv[0], lik[0], seqs[0].markers, 'default', 0.5, True, False, covs)
    g = out['pts'][0]
    np.testing.assert_array_equal(np.isnan(g), np.isnan(pts))
    m = ~np.isnan(pts)
    np.testing.assert_allclose(g[m], pts[m], rtol=0, atol=1e-7)
    xe = out['x_est'][0]
    # the initial state is fitted on SBA points that agree with the oracle's to ~4e-9 m; the
    # first 87-state update carries that into x_est[0] at the 1e-8 level
    np.testing.assert_allclose(xe[0], o['x_est'][0], rtol=0, atol=1e-7)
    np.testing.assert_allclose(xe[:, :P], o['x_est'][:, :P], rtol=0, atol=10 * TOL['x'])
    np.testing.assert_allclose(out['x_smooth'][0][:, :P], o['x_smooth'][:, :P], rtol=0, atol=10 * TOL['smoothed_x'])


def test_pipeline_rejects_sequence_without_nose(ctx):
    scene = synth.load_scene_file()
    q = synth.make_sequence(6, scene, mode='default_nolure', seed=5)
    lik = q.likelihood.copy()
    lik[:, :, 0] = 0.0                       # nose never above the threshold
    table = pkin.build_table('head')
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    with pytest.raises(RuntimeError, match='nose'):
        ctx.sba_ekf_pipeline(table, cams, q.uv[None], lik[None], q.markers, 90.0, 0.5, 2704.0,
                             cekf.measurement_std(6), cekf.process_covariance(6, 1 / 90.0),
                             cekf.initial_covariance('head'))
