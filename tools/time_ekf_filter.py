"""Filter-kernel latency per frame, for rocprofv3 --kernel-trace --stats (the kernels' own
durations, no profiling build): one sequence of N frames per configuration, each run twice
(the second is the timed one in the trace; k_ekf_filter* average / N = us per frame).
python tools/time_ekf_filter.py [N]   (configurations: head / default x 12 cams x fd / analytic)"""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

from acinoset_amd import _native, synth, kinematics as pkin  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ctx = _native.Context(0)
for mode, n_cams, jac in [('head', 12, 'fd'), ('head', 12, 'analytic'), ('default', 12, 'fd'),
                          ('default', 12, 'analytic')]:
    scene = synth.ring_scene(n_cams)
    seq = synth.make_sequence(N, scene, mode=mode, seed=5)
    table = pkin.build_table(mode)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    P = table.P
    covs = cekf.ring_cal_covs(n_cams)
    s0 = np.zeros((1, 3 * P))
    s0[0, :P] = seq.x[0]
    s0[0, P:2 * P] = (seq.x[1] - seq.x[0]) / seq.Ts
    for _ in range(2):
        out = ctx.ekf_run(table, cams, seq.uv[None], seq.likelihood[None], 90.0, 0.5, float(scene.res[0]),
                          cekf.measurement_std(n_cams, covs), cekf.process_covariance(P, 1 / 90.),
                          cekf.initial_covariance(mode), s0, ref_numerics=jac == 'fd', jacobian=jac)
    print(f'{mode} {n_cams} cams {jac}: {N} frames, outliers {int(out["outliers"][0])}', flush=True)
