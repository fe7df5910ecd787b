"""One bench-shaped EKF call (bench.py's `ekf` leg: 12-camera head model, 64 sequences x 500
frames, reference numerics) repeated, for rocprofv3 --kernel-trace: the split of a call
between the filter, the RTS gains and the smoothed-state recursion.
python tools/prof_ekf_call.py [mode] [n_seq] [frames] [reps]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

from acinoset_amd import _native, synth, kinematics as pkin  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
mode = sys.argv[1] if len(sys.argv) > 1 else 'head'
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
N = int(sys.argv[3]) if len(sys.argv) > 3 else 500
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
C = 12
ctx = _native.Context(0)
scene = synth.ring_scene(C)
seqs = [synth.make_sequence(N, scene, mode=mode, seed=100 + k) for k in range(S)]
table = pkin.build_table(mode)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
P = table.P
covs = cekf.ring_cal_covs(C)
s0 = np.zeros((S, 3 * P))
for k, q in enumerate(seqs):
    s0[k, :P] = q.x[0]
    s0[k, P:2 * P] = (q.x[1] - q.x[0]) / q.Ts
uv = np.stack([q.uv for q in seqs])
lik = np.stack([q.likelihood for q in seqs])
for _ in range(reps):
    out = ctx.ekf_run(table, cams, uv, lik, 90.0, 0.5, float(scene.res[0]), cekf.measurement_std(C, covs),
                      cekf.process_covariance(P, 1 / 90.), cekf.initial_covariance(mode), s0)
print(f'{mode}: {S} sequences x {N} frames, outliers {int(out["outliers"].sum())}')
