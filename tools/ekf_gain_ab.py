"""A/B of the EKF between two builds of the library: the filtered and smoothed states of a
12-camera ring clip (float64 and reference numerics), saved to OUT.npz. Run once per build
(ACINOSET_HIP_LIB=<lib> python tools/ekf_gain_ab.py OUT.npz [frames] [mode]; mode 'default' (the
RTS gains' A/B of round 5) or 'head') and compare the files with --compare A.npz B.npz
(bit-identical expected for a reorganised kernel)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

if sys.argv[1] == '--compare':
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        print(f'{k}: {"bit-identical" if same else "DIFFERENT"} max|diff| {np.abs(a[k] - b[k]).max():.3e}')
    sys.exit(0 if all(np.array_equal(a[k], b[k]) for k in a.files) else 1)

import importlib  # noqa: E402
from acinoset_amd import _native  # noqa: E402
from test_gpu_ekf import _setup_ring  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')  # the module (the package re-exports a function of that name)

frames = int(sys.argv[2]) if len(sys.argv) > 2 else 60
mode = sys.argv[3] if len(sys.argv) > 3 else 'default'
ctx = _native.Context(0)
scene, seq, s0, cp, covs = _setup_ring(mode, frames)
out = {}
for ref in (False, True):
    r = cekf.run(seq.uv, seq.likelihood, cp, mode, 90.0, s0, ref_numerics=ref, cal_covs=covs, ctx=ctx)
    out[f'x_smooth_ref{int(ref)}'] = r['x_smooth']
    out[f'x_est_ref{int(ref)}'] = r['x_est']
np.savez(sys.argv[1], **out)
print('saved', sys.argv[1], {k: v.shape for k, v in out.items()})
