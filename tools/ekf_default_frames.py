"""The 29-state default EKF model against the oracle frame by frame over its first frames
(where the reference's own run diverges, ~18 frames): 6-camera golden fixture and 12-camera
ring, reference numerics / float64 forward differences / float64 analytic H.
    python tools/ekf_default_frames.py [frames]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import numpy as np  # noqa: E402

from acinoset_amd import _native, synth  # noqa: E402
from oracle import ekf as oekf, fisheye, kinematics as okin  # noqa: E402
from conftest import golden  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ctx = _native.Context(0)
P = 29


def setups():
    g = golden('ekf_default')
    uv, lik = g['uv'][:N], g['likelihood'][:N]
    C, L = uv.shape[1], uv.shape[2]
    fr, ca, mk = np.meshgrid(np.arange(len(g['uv'])), np.arange(C), np.arange(L), indexing='ij')
    fr_, mk_, xyz = fisheye.pairwise_points(fr.ravel(), ca.ravel(), mk.ravel(), g['uv'][..., 0].ravel(),
                                            g['uv'][..., 1].ravel(), g['K'], g['D'], g['R'], g['t'])
    s0 = oekf.initial_state('default', fr_, mk_, xyz, 0, 1 / 90.0)
    yield '6cam-golden', uv, lik, (g['K'], g['D'], g['R'], g['t']), tuple(g['res']), 6, None, s0, g
    scene = synth.ring_scene(12)
    seq = synth.make_sequence(N, scene, mode='default', seed=61)
    valid = (seq.likelihood > 0.5) & np.isfinite(seq.uv).all(-1)
    fr, ca, mk = np.nonzero(valid)
    fr_, mk_, xyz = fisheye.pairwise_points(fr, ca, mk, seq.uv[fr, ca, mk, 0], seq.uv[fr, ca, mk, 1], scene.K,
                                            scene.D, scene.R, scene.t)
    s0 = oekf.initial_state('default', fr_, mk_, xyz, 0, 1 / 90.0)
    yield ('12cam-ring', seq.uv, seq.likelihood, (scene.K, scene.D, scene.R, scene.t), tuple(scene.res), 12,
           cekf.ring_cal_covs(12), s0, None)


for name, uv, lik, (K, D, R, t), res, nc, covs, s0, g in setups():
    cp = (K, D, R, t, res, nc)
    for ref, jac in ((True, 'fd'), (False, 'fd'), (False, 'analytic')):
        out = cekf.run(uv, lik, cp, 'default', 90.0, s0, ref_numerics=ref, cal_covs=covs, ctx=ctx, jacobian=jac)
        o = oekf.ekf(uv, lik, K, D, R, t, 'default', 90.0, s0, 0.5, float(res[0]), ref_numerics=ref, cal_covs=covs,
                     jacobian=jac)
        ex = np.abs(out['x_est'][:, :P] - o['x_est'][:, :P]).max(1)
        ep = np.abs(okin.marker_positions('default', out['x_est'][:, :P]) -
                    okin.marker_positions('default', o['x_est'][:, :P])).max(axis=(1, 2))
        extra = ''
        if g is not None and ref and jac == 'fd':
            er = np.abs(out['x_est'][:, :P] - g['out_x'][:N]).max(1)
            extra = ' | vs reference run: ' + ' '.join(f'{v:.1e}' for v in er)
        print(f'{name} ref={ref} {jac}: |x_gpu - x_oracle| per frame: ' + ' '.join(f'{v:.1e}' for v in ex), flush=True)
        print(f'   positions (m): ' + ' '.join(f'{v:.1e}' for v in ep) + extra, flush=True)
        print(f'   oracle |x| per frame: ' + ' '.join(f'{v:.1e}' for v in np.abs(o['x_est'][:, :P]).max(1)), flush=True)
