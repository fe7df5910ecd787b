"""Frame-window FTE and point-shard extrinsics SBA with more ranks than the work divides into
well: few frames per rank (N = 10 / 20 over 8 ranks), more ranks than points."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402

from oracle import fte as ofte  # noqa: E402
from acinoset_amd import _native, dist, kinematics as pkin, synth  # noqa: E402

ctx = _native.Context(0)
scene = synth.load_scene_file()
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
table = pkin.build_table('default_nolure')
for N, world in [(10, 8), (20, 8), (6, 4), (12, 8), (3, 8), (2, 4), (4, 16)]:
    try:
        seq = synth.make_sequence(N, scene, mode='default_nolure', seed=2, tau_max=0.004)
        w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
        prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                            intermode='vel')
        X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
        X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
        Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, world=world)
        print(f'fte N={N} world={world}: iters {rd["iters"]}/{r1["iters"]} status {rd["status"]}/{r1["status"]} '
              f'|X| {np.abs(Xd - X1).max():.2e} |tau| {np.abs(td - t1).max():.2e}', flush=True)
    except Exception as e:
        print(f'fte N={N} world={world}: EXC {e!r}'[:300], flush=True)

from test_gpu_sba_ext import _synthetic  # noqa: E402
for n_pts, world in [(5, 8), (3, 4), (40, 8)]:
    try:
        K, D, R0, t0, X0, uv, pi, ci = _synthetic(n_pts, 6, 3)
        c6 = _native.pack_cameras(K, D, R0, t0)
        o = ctx.sba_ext_opts(max_iters=20)
        c1, X1, _, _, r1 = ctx.sba_extrinsics(c6, uv, pi, ci, X0, o)
        out = dist.sba_extrinsics_virtual(ctx, c6, uv, pi, ci, X0, o, world=world)
        cd, Xd = out[0], out[1]
        print(f'sba_ext pts={n_pts} world={world}: |X| {np.abs(Xd - X1).max():.2e} |cams| {np.abs(cd - c1).max():.2e}',
              flush=True)
    except Exception as e:
        print(f'sba_ext pts={n_pts} world={world}: EXC {e!r}'[:300], flush=True)
