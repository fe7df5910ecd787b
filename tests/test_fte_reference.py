"""FTE problem definition pinned to the REFERENCE's own Pyomo model (src/core/fte.py).

`tests/golden/fte_*.npz` were written by `tests/golden/make_golden.py fte`, which ran the
reference's `core.fte.fte` up to the IPOPT call with a numeric Pyomo stand-in
(`tests/golden/_pyomo_eval.py`) and evaluated the reference's constraint and objective
rules at recorded points. What this pins (IPOPT itself is absent, so the optimiser is
still pinned only by the oracle):

* the constraint blocks the reference creates (its joint-angle bounds never are);
* the reference's initial point (:254-292) = `core.fte.initial_state`;
* the dense measurement / weight extraction (:195-225) = `core.fte.build_measurements`;
* every constraint body and the objective, term by term, at a random point;
* the exact elimination: at feasible points of the reference model, the reduced
  objective of `oracle/fte.py` (and of the GPU, `acs_fte_eval`) equals the reference
  objective, and the X / virtual-frame map reproduces the reference's x, dx, ddx;
* the output states (:540-555) = `core.fte.states_from_solution`.

Tolerances: objective 1e-11 relative; constraint bodies 1e-9 absolute (px, m, m/s);
dx / ddx from the virtual-frame map 1e-9 relative to their scale.
"""
import glob
import importlib
import os

import numpy as np
import pandas as pd
import pytest

from oracle import fte as ofte, kinematics as okin
from oracle.fisheye import project

cfte = importlib.import_module('acinoset_amd.core.fte')

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, 'fte_*.npz')))
EXPECTED = {'pose_constraint', 'measurement', 'integrate_p', 'integrate_v', 'constant_acc'}


def _load(name):
    z = np.load(os.path.join(HERE, name + '.npz'))
    return {k: z[k] for k in z.files}


def _dims(f):
    mode = str(f['mode'])
    N = int(f['end_frame'] - f['start_frame'] + 1)
    P = len(okin.POSE[mode])
    C = f['K'].shape[0]
    L = len(okin.marker_positions(mode, np.zeros((1, P)))[0])
    return mode, N, P, C, L


def _df(f, mode):
    from acinoset_amd.kinematics import get_markers
    markers = np.array(get_markers(mode), dtype=object)
    return pd.DataFrame({'frame': f['df_frame'], 'camera': f['df_camera'], 'marker': markers[f['df_marker']],
                         'x': f['df_x'], 'y': f['df_y'], 'likelihood': f['df_likelihood']})


def _tau(f, tag, N, C):
    if not bool(f['sd']):
        return np.zeros(C)
    t = f[f'{tag}_var_shutter_delay']
    return t.reshape(N, C) if str(f['sd_mode']) == 'variable' else t


def _X_from_reference(x, dx, ddx, Ts):
    """Virtual frames carrying the reference's free dx[1], ddx[1] (oracle/fte.py header)."""
    X0 = x[0] - Ts * dx[0]
    Xm1 = X0 - Ts * (dx[0] - Ts * ddx[0])
    return np.concatenate([Xm1[None], X0[None], x], 0)


def _problem(f):
    mode, N, P, C, L = _dims(f)
    meas, w = cfte.build_measurements(_df(f, mode), list(okin_markers(mode)), C, int(f['start_frame']),
                                      int(f['end_frame']), float(f['thresh']))
    sd = bool(f['sd'])
    return ofte.Problem(mode, meas, w, f['K'], f['D'], f['R'], f['t'], 1.0 / float(f['fps']), sd=sd,
                        intermode=str(f['intermode']), sd_mode=str(f['sd_mode'])), meas, w


def okin_markers(mode):
    from acinoset_amd.kinematics import get_markers
    return get_markers(mode)


def test_fixtures_present():
    assert len(CASES) >= 4, CASES


@pytest.mark.parametrize('name', CASES)
def test_reference_constraint_blocks(name):
    f = _load(name)
    got = set(str(c) for c in f['constraints'])
    want = EXPECTED | ({'shutter_base_constraint', 'shutter_delay_constraint'} if bool(f['sd']) else set())
    # the joint-angle bounds (src/core/fte.py:330-430) are gated on pose-parameter names
    # being in the marker list, so the reference never creates them
    assert got == want


@pytest.mark.parametrize('name', CASES)
def test_initial_point_matches_reference(name):
    f = _load(name)
    mode, N, P, C, L = _dims(f)
    nose = pd.DataFrame({'frame': f['nose_frame'], 'marker': 'nose', 'x': f['nose_xyz'][:, 0],
                         'y': f['nose_xyz'][:, 1], 'z': f['nose_xyz'][:, 2]})
    X0 = cfte.initial_state(nose, mode, int(f['start_frame']), int(f['end_frame']))
    np.testing.assert_allclose(X0[2:], f['init_x'].reshape(N, P), rtol=0, atol=1e-12)
    # dx = ddx = 0 at the reference's start <=> both virtual frames equal frame 1
    assert np.all(f['init_dx'] == 0) and np.all(f['init_ddx'] == 0)
    np.testing.assert_array_equal(X0[0], X0[2])
    np.testing.assert_array_equal(X0[1], X0[2])
    # poses initialised to FK(x) (:285-290), slack_meas and tau to 0
    pos = okin.marker_positions(mode, X0[2:])
    np.testing.assert_allclose(pos.ravel(), f['init_poses'], rtol=0, atol=1e-12)
    assert np.all(f['init_slack_meas'] == 0)
    if bool(f['sd']):
        assert np.all(f['init_shutter_delay'] == 0)


@pytest.mark.parametrize('name', CASES)
def test_measurements_match_reference_params(name):
    """The reference's meas / weight Params, recovered from its measurement-constraint
    bodies at the random point: body = proj - meas - slack, so meas = proj - slack - body."""
    f = _load(name)
    prob, meas, w = _problem(f)
    mode, N, P, C, L = _dims(f)
    x = f['rand_var_x'].reshape(N, P)
    poses = f['rand_var_poses'].reshape(N, L, 3)
    dx = f['rand_var_dx'].reshape(N, P)
    ddx = f['rand_var_ddx'].reshape(N, P)
    tau = prob.tau_frames(_tau(f, 'rand', N, C)) if bool(f['sd']) else np.zeros((N, C))
    body = f['rand_con_measurement'].reshape(N, C, L, 2)
    slack = f['rand_var_slack_meas'].reshape(N, C, L, 2)
    im = prob.im
    for c in range(C):
        pt = poses.copy()
        if im >= 1:
            pt = pt + (dx[:, :3] * tau[:, c, None])[:, None, :]
        if im == 2:
            pt = pt + (ddx[:, :3] * (tau[:, c, None] ** 2))[:, None, :]
        uv = project(pt.reshape(-1, 3), f['K'][c], f['D'][c], f['R'][c], f['t'][c], fte_form=True).reshape(N, L, 2)
        np.testing.assert_allclose(uv - slack[:, c] - body[:, c], meas[:, c], rtol=0, atol=1e-9)


@pytest.mark.parametrize('name', CASES)
def test_constraint_bodies_and_objective_at_random_point(name):
    f = _load(name)
    prob, meas, w = _problem(f)
    mode, N, P, C, L = _dims(f)
    Ts = prob.Ts
    v = {k: f[f'rand_var_{k}'] for k in ('x', 'dx', 'ddx', 'poses', 'slack_model', 'slack_meas')}
    x, dx, ddx = (v[k].reshape(N, P) for k in ('x', 'dx', 'ddx'))
    sm = v['slack_model'].reshape(N, P)
    # pose_constraint (:323-328): FK(x) - poses
    fk = okin.marker_positions(mode, x)
    np.testing.assert_allclose(f['rand_con_pose_constraint'], (fk.ravel() - v['poses']), rtol=0, atol=1e-12)
    # integration (:467-487), n >= 2
    np.testing.assert_allclose(f['rand_con_integrate_p'], (x[1:] - x[:-1] - Ts * dx[1:]).ravel(), atol=1e-12)
    np.testing.assert_allclose(f['rand_con_integrate_v'], (dx[1:] - dx[:-1] - Ts * ddx[1:]).ravel(), atol=1e-10)
    np.testing.assert_allclose(f['rand_con_constant_acc'], (ddx[1:] - ddx[:-1] - sm[1:]).ravel(), atol=1e-10)
    if bool(f['sd']):
        tau = _tau(f, 'rand', N, C)
        tf = prob.tau_frames(tau)
        np.testing.assert_allclose(f['rand_con_shutter_base_constraint'], tf[:, 0], atol=0)
        rng_ = f['rand_con_shutter_delay_constraint']          # (N*C, 3): lo, value, hi
        np.testing.assert_allclose(rng_[:, 1], tf.ravel(), atol=0)
        np.testing.assert_allclose(rng_[:, 0], -Ts, rtol=1e-15)
        np.testing.assert_allclose(rng_[:, 2], Ts, rtol=1e-15)
    # objective (:492-510): sum qinv * slack_model^2 + sum rho(w * slack_meas)
    rho = okin.redescending_loss(w[..., None] * v['slack_meas'].reshape(N, C, L, 2), 3.0, 10.0, 20.0)
    obj = rho.sum() + (prob.qinv * sm * sm).sum()
    np.testing.assert_allclose(obj, float(f['rand_obj']), rtol=1e-11)


@pytest.mark.parametrize('name', CASES)
def test_exact_elimination_at_feasible_points(name):
    """At feasible points of the reference model (integration and shutter constraints hold,
    poses / slacks from the reference's own bodies) the reduced objective of the oracle
    equals the reference objective: the elimination is exact."""
    f = _load(name)
    prob, meas, w = _problem(f)
    mode, N, P, C, L = _dims(f)
    Ts = prob.Ts
    for i in range(int(f['n_points'])):
        tag = f'pt{i}'
        x, dx, ddx = (f[f'{tag}_var_{k}'].reshape(N, P) for k in ('x', 'dx', 'ddx'))
        for k in ('integrate_p', 'integrate_v', 'constant_acc'):
            scale = {'integrate_p': 1.0, 'integrate_v': np.abs(dx).max(), 'constant_acc': np.abs(ddx).max()}[k]
            assert np.abs(f[f'{tag}_con_{k}']).max() <= 1e-12 * max(scale, 1.0) / Ts, k
        if bool(f['sd']):
            assert np.all(f[f'{tag}_con_shutter_base_constraint'] == 0)
            r = f[f'{tag}_con_shutter_delay_constraint']
            assert np.all((r[:, 0] <= r[:, 1]) & (r[:, 1] <= r[:, 2]))
        X = _X_from_reference(x, dx, ddx, Ts)
        xo, dxo, ddxo = prob.derivs(X)
        np.testing.assert_allclose(dxo, dx, rtol=0, atol=1e-9 * max(1.0, np.abs(dx).max()))
        np.testing.assert_allclose(ddxo, ddx, rtol=0, atol=1e-9 * max(1.0, np.abs(ddx).max()))
        tau = _tau(f, tag, N, C)
        F, Fm, Fq = prob.cost(X, tau)
        np.testing.assert_allclose(F, float(f[f'{tag}_obj']), rtol=1e-11)


@pytest.mark.parametrize('name', CASES)
def test_output_states_match_reference(name):
    """x, dx, ddx, shutter_delay the reference hands to save_fte (:540-555) at feasible
    point 0 = `core.fte.states_from_solution` of the reduced solution."""
    f = _load(name)
    mode, N, P, C, L = _dims(f)
    Ts = 1.0 / float(f['fps'])
    x, dx, ddx = (f[f'pt0_var_{k}'].reshape(N, P) for k in ('x', 'dx', 'ddx'))
    np.testing.assert_array_equal(f['out_x'], x)
    X = _X_from_reference(x, dx, ddx, Ts)
    tau = _tau(f, 'pt0', N, C)
    st = cfte.states_from_solution(X, tau, Ts, bool(f['sd']), N)
    np.testing.assert_allclose(np.array(st['x']), f['out_x'], rtol=0, atol=0)
    np.testing.assert_allclose(np.array(st['dx']), f['out_dx'], rtol=0, atol=1e-9 * max(1, np.abs(dx).max()))
    np.testing.assert_allclose(np.array(st['ddx']), f['out_ddx'], rtol=0, atol=1e-9 * max(1, np.abs(ddx).max()))
    if bool(f['sd']):
        np.testing.assert_array_equal(np.array(st['shutter_delay']), f['out_shutter_delay'])
    else:
        assert 'out_shutter_delay' not in f and 'shutter_delay' not in st
    assert int(f['out_start_frame']) == int(f['start_frame'])


@pytest.mark.gpu
@pytest.mark.parametrize('name', CASES)
def test_gpu_objective_equals_reference_objective(ctx, name):
    """acs_fte_eval at the reduced image of the reference's feasible points = the
    reference's own objective (1e-10 relative)."""
    from acinoset_amd import _native, kinematics as pkin
    f = _load(name)
    prob, meas, w = _problem(f)
    mode, N, P, C, L = _dims(f)
    cams = _native.pack_cameras(f['K'], f['D'], f['R'], f['t'])
    table = pkin.build_table(mode)
    for i in range(int(f['n_points'])):
        tag = f'pt{i}'
        x, dx, ddx = (f[f'{tag}_var_{k}'].reshape(N, P) for k in ('x', 'dx', 'ddx'))
        X = _X_from_reference(x, dx, ddx, prob.Ts)
        tau = _tau(f, tag, N, C)
        cost, g, H = ctx.fte_eval(table, cams, meas, w, prob.Ts, prob.qinv, X, tau, shutter_delay=prob.sd,
                                  intermode=prob.im, sd_mode=str(f['sd_mode']))
        np.testing.assert_allclose(cost[0], float(f[f'{tag}_obj']), rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize('name', CASES)
def test_gpu_reprojection_table_matches_reference(ctx, name):
    """The reprojection table the reference builds after its solve (:557-575,
    metric.residual_error) from feasible point 0, rebuilt by the drop-in's own
    post-processing (GPU FK + projection): frame and pixel_residual columns, 1e-9 px."""
    from acinoset_amd.lib import metric, misc
    f = _load(name)
    mode, N, P, C, L = _dims(f)
    Ts = 1.0 / float(f['fps'])
    x, dx, ddx = (f[f'pt0_var_{k}'].reshape(N, P) for k in ('x', 'dx', 'ddx'))
    X = _X_from_reference(x, dx, ddx, Ts)
    st = cfte.states_from_solution(X, _tau(f, 'pt0', N, C), Ts, bool(f['sd']), N)
    markers = list(okin_markers(mode))
    frames = np.arange(int(f['start_frame']), int(f['end_frame']) + 1)
    pos = misc.get_all_marker_coords_from_states(st, C, mode=mode, directions=True, intermode=str(f['intermode']))
    dfs = [pd.DataFrame({'frame': np.repeat(frames[None, :], L, 0).ravel(),
                         'marker': np.repeat(np.array(markers, dtype=object), N),
                         'x': p[:, :L, 0].T.ravel(), 'y': p[:, :L, 1].T.ravel(), 'z': p[:, :L, 2].T.ravel()})
           for p in pos]
    cam_params = (f['K'], f['D'], f['R'], f['t'], tuple(f['res']), C)
    err = metric.residual_error(_df(f, mode), dfs, markers, cam_params)
    for c in range(C):
        ref = f[f'out_reprj_{c}']
        got = err[str(c)][['frame', 'pixel_residual']].to_numpy(np.float64)
        np.testing.assert_array_equal(got[:, 0], ref[:, 0])
        np.testing.assert_allclose(got[:, 1], ref[:, 1], rtol=0, atol=1e-9)
