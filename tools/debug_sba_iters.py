"""Which points need the most LM iterations on the GPU (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from acinoset_amd import _native, synth
from oracle import sba as osba

ctx = _native.Context(0)
scene = synth.load_scene_file()
seq = synth.make_sequence(100, scene, mode='default_nolure', seed=0)
uv, mask, pts0, truth, _ = synth.dense_sba_problem(seq)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
prev = None
outs = {}
for k in range(1, 13):
    x, rep = ctx.sba_points_dense(cams, uv, mask, pts0, ctx.sba_opts(max_iters=k))
    outs[k] = x
    print(k, rep['status_counts'], flush=True)
full, _ = ctx.sba_points_dense(cams, uv, mask, pts0)
late = np.nonzero(np.any(outs[8] != full, axis=1))[0]
print('points still changing after 8 iterations:', late)
for p in late[:5]:
    ci = np.nonzero(mask[p])[0]
    print('point', p, 'cams', ci)
    for k in range(1, 13):
        print(' ', k, repr(outs[k][p]), np.abs(outs[k][p] - full[p]).max())
    xo, info = osba.sba_points(uv[p, ci], pts0[p:p + 1], np.zeros(len(ci), int), ci, scene.K, scene.D, scene.R,
                               scene.t, return_info=True)
    print('  oracle', repr(xo[0]), info['iters'], info['status'])
