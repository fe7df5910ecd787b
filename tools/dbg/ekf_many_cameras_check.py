"""EKF + RTS (the reference defines it for 'head' and 'default' only) on camera rings of 6 to
32 cameras against the oracle, float64: max |x_est - oracle| and |x_smooth - oracle| over the
first frames, and the marker-position difference."""
import importlib
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402

from oracle import ekf as oekf, kinematics as okin  # noqa: E402
from acinoset_amd import _native, kinematics as pkin  # noqa: E402
from test_gpu_ekf import _setup_ring  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
ctx = _native.Context(0)
CASES = [('head', 30, 6), ('head', 30, 16), ('head', 30, 24), ('head', 30, 32), ('default', 12, 16), ('default', 12, 24)]
if len(sys.argv) > 1 and sys.argv[1] == 'max':
    CASES = [('head', 10, 48), ('head', 10, 64), ('default', 4, 48), ('default', 4, 64)]
for mode, N, cams in CASES:
    try:
        scene, seq, s0, cp, covs = _setup_ring(mode, N, n_cams=cams)
        out = cekf.run(seq.uv, seq.likelihood, cp, mode, 90.0, s0, ref_numerics=False, cal_covs=covs,
                       covariances=True, ctx=ctx)
        o = oekf.ekf(seq.uv, seq.likelihood, scene.K, scene.D, scene.R, scene.t, mode, 90.0, s0, 0.5,
                     float(scene.res[0]), ref_numerics=False, cal_covs=covs)
        P = len(pkin.get_pose_params(mode))
        for n in (10, N):
            de = np.abs(out['x_est'][:n] - o['x_est'][:n]).max()
            ds = np.abs(out['x_smooth'][:n] - o['x_smooth'][:n]).max()
            dp = np.abs(okin.marker_positions(mode, out['x_smooth'][:n, :P]) -
                        okin.marker_positions(mode, o['x_smooth'][:n, :P])).max()
            print(f'{mode:15s} C={cams:2d} frames {n:3d}: |x_est| {de:.2e} |x_smooth| {ds:.2e} |pos| {dp:.2e} '
                  f'outliers {int(out["outliers"])}/{o["outliers"]}', flush=True)
    except Exception as e:
        print(f'{mode} C={cams}: ERROR {e!r}'[:400], flush=True)
