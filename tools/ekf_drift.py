"""GPU EKF vs the chained oracle over a configs[4] clip (bench_pipeline's rank-0 seed 3000 + k):
max |x_est - oracle| per 25-frame window, both numerics modes, for the EKF kernel in use
(ACS_EKF_WG=1 selects the 8-wave kernel for the head model too).
    python tools/ekf_drift.py [clip] [frames]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import numpy as np  # noqa: E402

from acinoset_amd import _native, kinematics as pkin, synth  # noqa: E402
from test_gpu_pipeline import _oracle  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
k = int(sys.argv[1]) if len(sys.argv) > 1 else 0
N = int(sys.argv[2]) if len(sys.argv) > 2 else 250
ctx = _native.Context(0)
scene = synth.ring_scene(12)
q = synth.make_sequence(N, scene, mode='default_nolure', seed=3000 + k)
table = pkin.build_table('head')
covs = cekf.ring_cal_covs(12)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
P = table.P
print(f'kernel: {"8-wave" if os.environ.get("ACS_EKF_WG") == "1" else "default dispatch"}, clip {k}, {N} frames')
for ref in (True, False):
    out = ctx.sba_ekf_pipeline(table, cams, q.uv[None], q.likelihood[None], q.markers, 90.0, 0.5,
                               float(scene.res[0]), cekf.measurement_std(12, covs), cekf.process_covariance(P, 1 / 90.0),
                               cekf.initial_covariance('head'), ref_numerics=ref)
    _, _, o = _oracle(scene, q.uv, q.likelihood, q.markers, 'head', 0.5, False, ref, covs)
    e = np.abs(out['x_est'][0] - o['x_est'])
    print(f'ref_numerics={ref}: outliers gpu {int(out["outliers"][0])} oracle {o["outliers"]}')
    for w0 in range(0, N, 25):
        sl = slice(w0, min(N, w0 + 25))
        print(f'  frames {w0:3d}-{sl.stop - 1:3d}: x {e[sl, :P].max():.2e} dx {e[sl, P:2 * P].max():.2e} '
              f'ddx {e[sl, 2 * P:].max():.2e}')
