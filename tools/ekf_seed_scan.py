"""Sensitivity of the 29-state default model's EKF on 12-camera ring clips: the oracle's
own run (float64, `jac` = analytic or fd) from s0 and from s0 (1 + 1e-12), and the largest
marker-position difference that rounding-level change grows to, per seed. The GPU and the
oracle differ by rounding, so a clip whose 1e-12 perturbation stays ~1e-6 m can be held to
north_star's 1e-4 m. python tools/ekf_seed_scan.py N fd|analytic seed [seed ...]
(profiles/r05/ekf_seed_scan.log)."""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from acinoset_amd import synth
from oracle import ekf as oe, fisheye, kinematics as okin
cekf = importlib.import_module('acinoset_amd.core.ekf')
mode='default'; N=int(sys.argv[1]); jac=sys.argv[2]; seeds=[int(s) for s in sys.argv[3:]]
scene = synth.ring_scene(12)
for seed in seeds:
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed)
    uv, lik = seq.uv, seq.likelihood
    valid = (lik > 0.5) & np.isfinite(uv).all(-1)
    fr, ca, mk = np.nonzero(valid)
    fr_, mk_, xyz = fisheye.pairwise_points(fr, ca, mk, uv[fr, ca, mk, 0], uv[fr, ca, mk, 1], scene.K, scene.D, scene.R, scene.t)
    s0 = oe.initial_state(mode, fr_, mk_, xyz, 0, 1 / 90.0)
    run = lambda s: oe.ekf(uv, lik, scene.K, scene.D, scene.R, scene.t, mode, 90.0, s, 0.5, float(scene.res[0]), ref_numerics=False, cal_covs=cekf.ring_cal_covs(12), jacobian=jac)
    a = run(s0); b = run(s0 * (1 + 1e-12))
    for key in ('x_est','x_smooth'):
        d = np.abs(okin.marker_positions(mode, a[key][:, :29]) - okin.marker_positions(mode, b[key][:, :29])).max(axis=(1,2))
        print(seed, N, jac, key, 'max pos diff per 3 frames', ' '.join(f'{x:.0e}' for x in d[::3]), 'max', f'{d.max():.1e}', flush=True)
