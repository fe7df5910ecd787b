"""GPU EKF against the oracle over whole clips (verdict r04 #3): the per-clip / per-window
maxima that the whole-clip parity tests' bounds are set from.

A. configs[4]: the bench's pipeline step (80 clips x 250 frames, 12-camera ring, head model),
   both numerics, the oracle chained on `n_oracle` clips: max |x_est|, |x_smooth| per state
   block and the marker positions (FK of x_est / x_smooth) against the oracle's.
B. 12-camera ring through core.ekf.run (acs_ekf_run), head and default models, reference
   numerics / float64 / analytic H, per 25-frame window.
    python tools/ekf_drift_survey.py [n_oracle] [frames]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import numpy as np  # noqa: E402

from acinoset_amd import _native, kinematics as pkin, synth  # noqa: E402
from oracle import ekf as oekf, fisheye, kinematics as okin  # noqa: E402
from test_gpu_pipeline import _oracle  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
n_or = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 250
ctx = _native.Context(0)


def pos(mode, x):
    return okin.marker_positions(mode, x)


def blocks(a, b, P):
    e = np.abs(a - b)
    return e[:, :P].max(), e[:, P:2 * P].max(), e[:, 2 * P:].max()


print(f'== A. configs[4] pipeline, 80 clips x {N} frames, 12 cams, head; oracle on {n_or} clips', flush=True)
scene = synth.ring_scene(12)
seqs = [synth.make_sequence(N, scene, mode='default_nolure', seed=3000 + k) for k in range(80)]
uv = np.stack([q.uv for q in seqs])
lik = np.stack([q.likelihood for q in seqs])
table = pkin.build_table('head')
covs = cekf.ring_cal_covs(12)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
P = table.P
for ref in (True, False):
    out = ctx.sba_ekf_pipeline(table, cams, uv, lik, seqs[0].markers, 90.0, 0.5, float(scene.res[0]),
                               cekf.measurement_std(12, covs), cekf.process_covariance(P, 1 / 90.0),
                               cekf.initial_covariance('head'), ref_numerics=ref)
    worst = np.zeros(7)
    for k in np.random.default_rng(2024).choice(80, n_or, replace=False):
        _, _, o = _oracle(scene, uv[k], lik[k], seqs[k].markers, 'head', 0.5, False, ref, covs)
        xe, xs = out['x_est'][k], out['x_smooth'][k]
        be = blocks(xe, o['x_est'], P)
        bs = blocks(xs, o['x_smooth'], P)
        pe = np.abs(pos('head', xe[:, :P]) - pos('head', o['x_est'][:, :P])).max()
        ps = np.abs(pos('head', xs[:, :P]) - pos('head', o['x_smooth'][:, :P])).max()
        row = np.array([*be, *bs[:1], pe, ps, abs(int(out['outliers'][k]) - o['outliers'])])
        worst = np.maximum(worst, row)
        print(f'  ref={ref!s:5} clip {k:2d}: x {be[0]:.2e} dx {be[1]:.2e} ddx {be[2]:.2e} | xs {bs[0]:.2e} | '
              f'pos_est {pe:.2e} m pos_smooth {ps:.2e} m | outliers d{int(row[-1])}', flush=True)
    print(f'  ref={ref!s:5} WORST: x {worst[0]:.2e} dx {worst[1]:.2e} ddx {worst[2]:.2e} xs {worst[3]:.2e} '
          f'pos_est {worst[4]:.2e} pos_smooth {worst[5]:.2e} outliers d{int(worst[6])}', flush=True)

print(f'== B. 12-cam ring, core.ekf.run, {N} frames, per 25-frame window', flush=True)
for mode in ('head', 'default'):
    scene = synth.ring_scene(12)
    seq = synth.make_sequence(N, scene, mode=mode, seed=61)
    valid = (seq.likelihood > 0.5) & np.isfinite(seq.uv).all(-1)
    fr, ca, mk = np.nonzero(valid)
    fr_, mk_, xyz = fisheye.pairwise_points(fr, ca, mk, seq.uv[fr, ca, mk, 0], seq.uv[fr, ca, mk, 1], scene.K,
                                            scene.D, scene.R, scene.t)
    s0 = oekf.initial_state(mode, fr_, mk_, xyz, 0, 1 / 90.0)
    cp = (scene.K, scene.D, scene.R, scene.t, tuple(scene.res), 12)
    covs = cekf.ring_cal_covs(12)
    P = len(pkin.get_pose_params(mode))
    for ref, jac in ((True, 'fd'), (False, 'fd'), (False, 'analytic')):
        try:
            out = cekf.run(seq.uv, seq.likelihood, cp, mode, 90.0, s0, ref_numerics=ref, cal_covs=covs, ctx=ctx,
                           jacobian=jac)
        except Exception as e:  # noqa: BLE001
            print(f'  {mode} ref={ref} {jac}: GPU error {e}', flush=True)
            continue
        o = oekf.ekf(seq.uv, seq.likelihood, scene.K, scene.D, scene.R, scene.t, mode, 90.0, s0, 0.5,
                     float(scene.res[0]), ref_numerics=ref, cal_covs=covs, jacobian=jac)
        print(f'  {mode} ref={ref} {jac}: outliers gpu {int(out["outliers"])} oracle {o["outliers"]}; '
              f'|x| max {np.abs(o["x_est"][:, :P]).max():.2e}', flush=True)
        pe = np.abs(pos(mode, out['x_est'][:, :P]) - pos(mode, o['x_est'][:, :P])).max(axis=(1, 2))
        ps = np.abs(pos(mode, out['x_smooth'][:, :P]) - pos(mode, o['x_smooth'][:, :P])).max(axis=(1, 2))
        for w0 in range(0, N, 25):
            sl = slice(w0, min(N, w0 + 25))
            be = blocks(out['x_est'][sl], o['x_est'][sl], P)
            bs = np.abs(out['x_smooth'][sl, :P] - o['x_smooth'][sl, :P]).max()
            print(f'    frames {w0:3d}-{sl.stop - 1:3d}: x {be[0]:.2e} dx {be[1]:.2e} ddx {be[2]:.2e} xs {bs:.2e} '
                  f'pos_est {pe[sl].max():.2e} pos_smooth {ps[sl].max():.2e}', flush=True)
