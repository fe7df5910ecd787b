"""A/B of the dense pairwise triangulation (acs_triangulate_dense) between two builds of the
library: a 12-camera ring clip's points saved to OUT.npz (ACINOSET_HIP_LIB=<lib> python
tools/tri_ab.py OUT.npz), compared with --compare A.npz B.npz (bit-identical expected)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))

if sys.argv[1] == '--compare':
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    ok = all(np.array_equal(a[k], b[k], equal_nan=True) for k in a.files)
    for k in a.files:
        print(f'{k}: {"bit-identical" if np.array_equal(a[k], b[k], equal_nan=True) else "DIFFERENT"}')
    sys.exit(0 if ok else 1)

from acinoset_amd import _native, synth  # noqa: E402

ctx = _native.Context(0)
scene = synth.ring_scene(12)
seq = synth.make_sequence(200, scene, seed=4242)
N, C, L, _ = seq.uv.shape
uv = np.ascontiguousarray(seq.uv.transpose(0, 2, 1, 3).reshape(N * L, C, 2))
mk = np.ascontiguousarray((seq.likelihood > 0.5).transpose(0, 2, 1).reshape(N * L, C))
xyz, cnt = ctx.triangulate_dense(_native.pack_cameras(scene.K, scene.D, scene.R, scene.t), uv, mk)
np.savez(sys.argv[1], xyz=xyz, cnt=cnt)
print('saved', sys.argv[1], xyz.shape)
