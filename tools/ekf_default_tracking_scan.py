"""Does any gentle synthetic workload let the 29-state default-model EKF (the reference's P0 / Q / R,
src/core/ekf.py:154-213) track, so that GPU = oracle could be pinned over a whole clip?
Oracle runs (float64, analytic H) from s0 and s0 (1 + 1e-12): smoothed marker RMS vs the truth and the
largest marker-position difference the 1e-12 change grows to, per 10 frames, for smaller gait
amplitudes / drift / speeds and several seeds. python tools/ekf_default_tracking_scan.py N n_cams"""
import sys, numpy as np, importlib, time
sys.path.insert(0,'/root/repo')
from acinoset_amd import synth
from oracle import ekf as oe, fisheye, kinematics as okin
cekf = importlib.import_module('acinoset_amd.core.ekf')
mode='default'
N=int(sys.argv[1]); ncam=int(sys.argv[2])
scene = synth.load_scene_file() if ncam == 6 else synth.ring_scene(ncam)
covs = None if ncam == 6 else cekf.ring_cal_covs(ncam)
cfgs = [(0.02,0.1,1.0,65),(0.02,0.1,0.5,65),(0.01,0.05,0.5,65),(0.02,0.1,1.0,61),(0.02,0.1,1.0,7)]
for ga, dr, sp, seed in cfgs:
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed, gait_amp=ga, drift=dr, speed=sp)
    uv, lik = seq.uv, seq.likelihood
    valid = (lik > 0.5) & np.isfinite(uv).all(-1)
    fr, ca, mk = np.nonzero(valid)
    fr_, mk_, xyz = fisheye.pairwise_points(fr, ca, mk, uv[fr, ca, mk, 0], uv[fr, ca, mk, 1], scene.K, scene.D, scene.R, scene.t)
    s0 = oe.initial_state(mode, fr_, mk_, xyz, 0, 1 / 90.0)
    t0=time.time()
    run = lambda s: oe.ekf(uv, lik, scene.K, scene.D, scene.R, scene.t, mode, 90.0, s, 0.5, float(scene.res[0]), ref_numerics=False, cal_covs=covs, jacobian='analytic')
    a = run(s0); b = run(s0*(1+1e-12))
    truth = okin.marker_positions(mode, seq.x)
    pe = okin.marker_positions(mode, a['x_smooth'][:, :29])
    err = np.sqrt(np.mean(np.sum((pe-truth)**2,-1),-1))
    d = np.abs(okin.marker_positions(mode, a['x_est'][:, :29]) - okin.marker_positions(mode, b['x_est'][:, :29])).max(axis=(1,2))
    print(f'cams={ncam} ga={ga} drift={dr} speed={sp} seed={seed}: smoothed rms/10fr', ' '.join(f'{x:.3f}' for x in err[::10]), '| sens per 10fr', ' '.join(f'{x:.0e}' for x in d[::10]), f'{time.time()-t0:.0f}s', flush=True)
