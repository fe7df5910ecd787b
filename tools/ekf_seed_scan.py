"""How long the 29-state default model keeps the synthetic subject of a 12-camera ring clip:
the oracle's own EKF (analytic H, float64) per seed, and the first frame whose state norm
departs from frame 0's by more than 10 %. python tools/ekf_seed_scan.py N seed [seed ...]
(profiles/r05/ekf_seed_scan.log: seed 62 tracks 28 of 30 frames, seed 61 14)."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from acinoset_amd import synth
from oracle import ekf as oe, fisheye
cekf = importlib.import_module('acinoset_amd.core.ekf')
mode='default'; N=int(sys.argv[1]); seeds=[int(s) for s in sys.argv[2:]]
scene = synth.ring_scene(12)
for seed in seeds:
    t0=time.time()
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed)
    uv, lik = seq.uv, seq.likelihood
    valid = (lik > 0.5) & np.isfinite(uv).all(-1)
    fr, ca, mk = np.nonzero(valid)
    fr_, mk_, xyz = fisheye.pairwise_points(fr, ca, mk, uv[fr, ca, mk, 0], uv[fr, ca, mk, 1], scene.K, scene.D, scene.R, scene.t)
    s0 = oe.initial_state(mode, fr_, mk_, xyz, 0, 1 / 90.0)
    o = oe.ekf(uv, lik, scene.K, scene.D, scene.R, scene.t, mode, 90.0, s0, 0.5, float(scene.res[0]), ref_numerics=False, cal_covs=cekf.ring_cal_covs(12), jacobian='analytic')
    nx = np.linalg.norm(o['x_est'][:, :29], axis=1)
    dep = np.nonzero(np.abs(nx - nx[0]) > 0.1 * nx[0])[0]
    print(seed, 'first departing frame', dep[0] if len(dep) else None, 'norms', np.round(nx[::3],1), f'{time.time()-t0:.0f}s', flush=True)
