"""EKF throughput probe (diagnostic)."""
import sys
import time
import importlib
import numpy as np
sys.path.insert(0, '.')
from acinoset_amd import _native, synth, kinematics as pkin

cekf = importlib.import_module('acinoset_amd.core.ekf')
ctx = _native.Context(0)
for mode, N, S, C in [('head', 1000, 1, 6), ('default', 1000, 1, 6), ('default', 1000, 64, 6), ('default', 2000, 1, 12)]:
    scene = synth.load_scene_file() if C == 6 else synth.ring_scene(C)
    seq = synth.make_sequence(N, scene, mode=mode, seed=5)
    table = pkin.build_table(mode)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    P = table.P
    s0 = np.zeros(3 * P)
    s0[:3] = seq.pos3d[0, 0, 0]
    meas = np.stack([seq.uv] * S)
    lik = np.stack([seq.likelihood] * S)
    covs = cekf.CAL_COVS if C == 6 else cekf.CAL_COVS * 2
    args = (90.0, 0.5, 2704.0, cekf.measurement_std(C, covs), cekf.process_covariance(P, 1 / 90.0),
            cekf.initial_covariance(mode))
    ctx.ekf_run(table, cams, meas[:, :20], lik[:, :20], *args, np.stack([s0] * S))
    t = time.perf_counter()
    out = ctx.ekf_run(table, cams, meas, lik, *args, np.stack([s0] * S))
    dt = time.perf_counter() - t
    print(f'{mode} N={N} seqs={S} C={C}: {dt*1e3:.1f} ms, {dt/N*1e6:.1f} us/frame/seq, {S*N/dt:.0f} frames/s', flush=True)
