"""Per-iteration comparison of the GPU extrinsics SBA with the oracle (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from conftest import golden
from oracle import sba_ext as oext
from acinoset_amd import _native

g = golden('sba_extrinsics')
ctx = _native.Context(0)
cams = _native.pack_cameras(g['K'], g['D'], g['R0'], g['t0'])
for k in list(range(1, 50)) + [200]:
    c, X, rb, ra, rep = ctx.sba_extrinsics(cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                           g['points_3d'], ctx.sba_ext_opts(max_iters=k))
    Xo, Ro, to, info = oext.sba_extrinsics(g['points_2d'], g['points_3d'], g['point_indices'].astype(np.int64),
                                           g['camera_indices'].astype(np.int64), g['K'], g['D'].reshape(-1, 4),
                                           g['R0'], g['t0'], max_iters=k)
    ro = oext.residuals(Xo, Ro, to, g['K'], g['D'].reshape(-1, 4), g['points_2d'], g['point_indices'],
                        g['camera_indices']).ravel()
    print(k, rep['iters'], info['iters'], rep['n_accepted'], info['n_accepted'], f"{rep['cost_after']:.12e}",
          f"{info['cost_after']:.12e}", f"{rep['lambda_final']:.1e}", f"{info['lam']:.1e}",
          f"{np.abs(ra - ro).max():.2e}", f"{np.abs(X - Xo).max():.2e}", rep['status_name'], info['status'],
          flush=True)
