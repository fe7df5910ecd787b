"""API edge behaviours on the GPU next to the oracle's: FTE max_iters = 0 and an all-zero-weight
frame; EKF on a clip whose likelihoods are all below the threshold; SBA points with every
observation masked."""
import importlib
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np  # noqa: E402

from oracle import fte as ofte, ekf as oekf  # noqa: E402
from acinoset_amd import _native, kinematics as pkin, synth  # noqa: E402

ctx = _native.Context(0)


def run(name, fn):
    try:
        print(name, '->', fn(), flush=True)
    except Exception as e:
        print(name, '-> EXC', repr(e)[:300], flush=True)


scene = synth.load_scene_file()
seq = synth.make_sequence(20, scene, mode='default_nolure', seed=2, tau_max=0.004)
w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True, intermode='vel')
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
X0 = ofte.initial_state(prob, np.arange(20), seq.pos3d[:, 0, 0])
table = pkin.build_table('default_nolure')


def fte0():
    X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                opts=ctx.fte_default_opts(max_iters=0))
    Xo, to, info = ofte.solve(prob, X0, max_iters=0)
    return (rep['status_name'], rep['iters'], float(np.abs(X - X0).max()), info['status'], info['iters'],
            float(np.abs(Xo - X0).max()), rep['cost_after'], info['cost_after'])


def fte_empty_frame():
    w2 = prob.w.copy()
    w2[5] = 0.0
    w2[6] = 0.0
    p2 = ofte.Problem('default_nolure', seq.uv, w2, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                      intermode='vel')
    X, tau, rep = ctx.fte_solve(table, cams, p2.meas, p2.w, p2.Ts, p2.qinv, X0)
    Xo, to, info = ofte.solve(p2, X0)
    return (rep['status_name'], rep['iters'], info['status'], info['iters'], float(np.abs(X - Xo).max()),
            abs(rep['cost_after'] - info['cost_after']) / info['cost_after'])


run('fte max_iters=0', fte0)
run('fte two frames without observations', fte_empty_frame)

cekf = importlib.import_module('acinoset_amd.core.ekf')
from test_gpu_ekf import _setup_ring  # noqa: E402


def ekf_blind():
    sc, sq, s0, cp, covs = _setup_ring('head', 10)
    lik = sq.likelihood.copy()
    lik[3:6] = 0.0   # frames 3-5: nothing above the threshold
    out = cekf.run(sq.uv, lik, cp, 'head', 90.0, s0, ref_numerics=False, cal_covs=covs, ctx=ctx)
    o = oekf.ekf(sq.uv, lik, sc.K, sc.D, sc.R, sc.t, 'head', 90.0, s0, 0.5, float(sc.res[0]), ref_numerics=False,
                 cal_covs=covs)
    return (float(np.abs(out['x_est'] - o['x_est']).max()), float(np.abs(out['x_smooth'] - o['x_smooth']).max()),
            int(out['outliers']), o['outliers'], bool(np.isfinite(out['x_smooth']).all()))


run('ekf frames 3-5 below threshold', ekf_blind)


def sba_all_masked():
    n = 50
    uv = np.zeros((n, 6, 2))
    mk = np.zeros((n, 6), np.uint8)
    X0 = np.random.default_rng(0).normal(size=(n, 3))
    out = ctx.sba_points_dense(cams, uv, mk, X0) if hasattr(ctx, 'sba_points_dense') else None
    return 'no dense API' if out is None else (float(np.abs(out[0] - X0).max()), out[-1] if len(out) > 1 else None)


run('sba all observations masked', sba_all_masked)
