"""One LM step of the FTE solve (GPU vs oracle) on ring scenes of several camera counts and
modes: max |X - Xo|, |tau - to|, and the eval (cost, gradient, normal matrix) at X0."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from oracle import fte as ofte  # noqa: E402
from acinoset_amd import _native, kinematics as pkin, synth  # noqa: E402

ctx = _native.Context(0)
for n_cams, mode, N, sdm, inter in [(16, 'default_nolure', 31, 'const', 'pos'), (16, 'default_nolure', 31, 'const', 'acc'),
                                    (16, 'default', 31, 'const', 'acc')] + [(*c, 'vel') for c in [(6, 'default_nolure', 7, 'const'), (12, 'default_nolure', 7, 'const'),
                             (15, 'default_nolure', 7, 'const'), (16, 'default_nolure', 7, 'const'),
                             (16, 'default_nolure', 7, 'none'), (12, 'default', 7, 'const'),
                             (16, 'default', 7, 'const'), (16, 'default_nolure', 31, 'const'),
                             (16, 'default_nolure', 400, 'const'), (12, 'default_nolure', 400, 'const'),
                             (16, 'head', 400, 'const'), (16, 'default', 200, 'const')]]:
    scene = synth.ring_scene(n_cams) if n_cams != 6 else synth.load_scene_file()
    sd = sdm != 'none'
    seq = synth.make_sequence(N, scene, mode=mode, seed=2, tau_max=0.004 if sd else 0.0)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem(mode, seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=sd, intermode=inter,
                        sd_mode='const')
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    table = pkin.build_table(mode)
    tau0 = np.zeros(n_cams)
    try:
        c, g, H = ctx.fte_eval(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, tau0, shutter_delay=sd,
                               intermode=prob.im)
        co = prob.cost(X0, tau0 if sd else np.zeros(n_cams))[0]
        c = float(np.ravel(np.asarray(c, dtype=float))[0])
        g, H = np.asarray(g), np.asarray(H)
        Fo, Ho, go = prob.linearize(X0, tau0 if sd else np.zeros(n_cams))
        go = go.copy()
        if sd:
            go[prob.M * prob.P] = 0.0
        Ho = Ho.toarray()
        ev = f'eval: cost {abs(c - co) / abs(co):.1e} g {float(np.abs(g - go).max() / np.abs(go).max()):.1e} ' \
             f'H {float(np.abs(H - Ho).max() / np.abs(Ho).max()):.1e}'
        X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, shutter_delay=sd,
                                    intermode=prob.im, opts=ctx.fte_default_opts(max_iters=1))
        Xo, to, info = ofte.solve(prob, X0, max_iters=1)
        dt = float(np.abs(np.asarray(tau) - np.asarray(to)).max()) if sd else 0.0
        print(f'C={n_cams:2d} {mode:15s} N={N:3d} sd={sdm:5s} {inter}: step |X-Xo| {float(np.abs(X - Xo).max()):.2e} '
              f'|tau-to| {dt:.2e} bad {rep["n_bad_pivots"]} acc {rep["n_accepted"]}/{info["n_accepted"]} {ev}',
              flush=True)
    except Exception as e:
        print(f'C={n_cams} {mode} N={N}: ERROR {e!r}'[:300], flush=True)
