import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from acinoset_amd import _native, workloads
from oracle import sba as osba
ctx = _native.Context(0)
wl = workloads.sba_reference_workload()
opts = ctx.sba_opts()
pd_, rep = ctx.sba_points_dense(wl.cams, wl.uv, wl.mask, wl.pts0, opts)
pl, rb, ra, repl = ctx.sba_points(wl.cams, wl.points_2d, wl.point_idx, wl.cam_idx, wl.pts0, opts)
po = osba.sba_points(wl.points_2d, wl.pts0, wl.point_idx, wl.cam_idx, wl.K, wl.D, wl.R, wl.t)
e_d = np.linalg.norm(pd_ - po, axis=1); e_l = np.linalg.norm(pl - po, axis=1)
print('dense rep', rep); print('list rep', repl)
print('dense vs oracle max', e_d.max(), 'n>1e-6', (e_d > 1e-6).sum()); print('list vs oracle max', e_l.max())
bad = np.argsort(-e_d)[:8]
for i in bad:
    print(i, e_d[i], wl.pts0[i], po[i], pd_[i], wl.mask[i], wl.uv[i].tolist())
# same problem through the dense kernel with the oracle's own start for comparison
print('cams', wl.cams.shape, wl.cams.dtype, wl.uv.dtype, wl.mask.dtype, wl.uv.flags['C_CONTIGUOUS'], wl.mask.flags['C_CONTIGUOUS'])
