"""N = 2 frame windows over 2-4 ranks: the single-GPU and the distributed iterates after 1, 5,
20 and all LM steps (where do they separate?)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import fte as ofte  # noqa: E402
from acinoset_amd import _native, dist, kinematics as pkin, synth  # noqa: E402

ctx = _native.Context(0)
scene = synth.load_scene_file()
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
table = pkin.build_table('default_nolure')
N = 2
seq = synth.make_sequence(N, scene, mode='default_nolure', seed=2, tau_max=0.004)
w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True, intermode='vel')
X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
for world in (2, 3, 4):
    for it in (1, 5, 20, 40, 200):
        o = ctx.fte_default_opts(max_iters=it)
        X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, opts=o)
        Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, opts=o,
                                            world=world)
        Xo, to, io = ofte.solve(prob, X0, max_iters=it)
        print(f'world {world} max_iters {it:3d}: single {r1["iters"]}/{r1["n_accepted"]} dist {rd["iters"]}/'
              f'{rd["n_accepted"]} oracle {io["iters"]}/{io["n_accepted"]} |Xd-X1| {np.abs(Xd - X1).max():.2e} '
              f'|X1-Xo| {np.abs(X1 - Xo).max():.2e} cost {r1["cost_after"]:.10g} {rd["cost_after"]:.10g} '
              f'{io["cost_after"]:.10g}', flush=True)
