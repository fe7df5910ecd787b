"""`core.fte` (src/core/fte.py:28-588) with the Pyomo model + IPOPT solve replaced by the
GPU trajectory solve (acs_fte_solve, acinoset_amd/csrc/fte.hip).

Kept from the reference: the signature and option checks (:28-48), the redescending
loss knots (:53-55), R and the Q table (:112-144), the reconstruction_params.json dump
(:148-160), pairwise-triangulation + linear-regression initialisation (:165-170,
:254-292), the measurement weights (:210-215), the output states (x, dx, ddx,
shutter_delay; :540-555), the reprojection table (:557-575) and fte.pickle (:579).
Not reproduced: IPOPT options/logging, PDF plots, labelled videos.
"""
import json
import os
from time import time
from typing import Dict

import numpy as np

from .. import _native
from ..kinematics import build_table, get_markers, get_pose_params
from ..lib import app, metric, misc, utils

REDESC_A, REDESC_B, REDESC_C = 3, 10, 20
R_MEAS = 3
Q_TABLE = {'x_0': 4, 'y_0': 7, 'z_0': 5, 'phi_0': 13, 'theta_0': 9, 'psi_0': 26, 'l_1': 4, 'phi_1': 32,
           'theta_1': 18, 'psi_1': 12, 'theta_2': 43, 'phi_3': 10, 'theta_3': 53, 'psi_3': 34, 'theta_4': 90,
           'psi_4': 43, 'theta_5': 118, 'psi_5': 51, 'theta_6': 247, 'theta_7': 186, 'theta_8': 194,
           'theta_9': 164, 'theta_10': 295, 'theta_11': 243, 'theta_12': 334, 'theta_13': 149, 'x_l': 4,
           'y_l': 7, 'z_l': 5}
INTERMODES = {'pos': 0, 'vel': 1, 'acc': 2}


def model_weights(mode):
    """1/Q with Q = _Q^2 (src/core/fte.py:144, :217-218)."""
    return np.array([1.0 / float(Q_TABLE[p]) ** 2 for p in get_pose_params(mode)])


def build_measurements(points_2d_df, markers, n_cams, start_frame, end_frame, dlc_thresh, R=R_MEAS):
    """Dense (N, C, L, 2) measurements and (N, C, L) weights: 1/R where likelihood >
    thresh else 0 (src/core/fte.py:195-225; the first matching row wins, as `.values[0]`)."""
    N, L = end_frame - start_frame + 1, len(markers)
    meas = np.zeros((N, n_cams, L, 2))
    w = np.zeros((N, n_cams, L))
    mi = {m: i for i, m in enumerate(markers)}
    df = points_2d_df[points_2d_df['frame'].between(start_frame, end_frame) & points_2d_df['marker'].isin(markers)]
    df = df.drop_duplicates(subset=['frame', 'camera', 'marker'], keep='first')
    n = df['frame'].to_numpy().astype(int) - start_frame
    c = df['camera'].to_numpy().astype(int)
    ok = (c >= 0) & (c < n_cams)
    n, c = n[ok], c[ok]
    l_ = np.array([mi[m] for m in df['marker'][ok]], dtype=int)
    meas[n, c, l_, 0] = df['x'].to_numpy()[ok]
    meas[n, c, l_, 1] = df['y'].to_numpy()[ok]
    w[n, c, l_] = np.where(df['likelihood'].to_numpy()[ok] > dlc_thresh, 1.0 / R, 0.0)
    meas = np.nan_to_num(meas)
    return meas, w


def initial_state(points_3d_df, mode, start_frame, end_frame):
    """src/core/fte.py:254-292: least-squares line of the triangulated nose over absolute
    frame numbers -> x_0, y_0, z_0; psi_0 = atan2(y_slope, x_slope); the rest 0; dx = ddx
    = 0, i.e. both virtual frames equal the first frame. Returns X (N+2, P)."""
    idx = get_pose_params(mode)
    P, N = len(idx), end_frame - start_frame + 1
    nose = points_3d_df[points_3d_df['marker'] == 'nose'][['frame', 'x', 'y', 'z']].to_numpy(np.float64)
    if len(nose) < 2:
        raise ValueError('FTE initialisation needs the nose triangulated in at least two frames')
    fr = nose[:, 0]
    A = np.stack([fr, np.ones_like(fr)], 1)
    (sx, ix), (sy, iy), (sz, iz) = (np.linalg.lstsq(A, nose[:, j], rcond=None)[0] for j in (1, 2, 3))
    f = np.arange(start_frame, end_frame + 1, dtype=np.float64)
    x = np.zeros((N, P))
    x[:, idx['x_0']] = f * sx + ix
    x[:, idx['y_0']] = f * sy + iy
    x[:, idx['z_0']] = f * sz + iz
    x[:, idx['psi_0']] = np.arctan2(sy, sx)
    return np.concatenate([x[:1], x[:1], x], 0)


def states_from_solution(X, tau, Ts, shutter_delay, N):
    """x, dx, ddx (N x P lists) and shutter_delay (C lists of N) as src/core/fte.py:540-555."""
    x = X[2:]
    dx = (X[2:] - X[1:-1]) / Ts
    ddx = (X[2:] - 2 * X[1:-1] + X[:-2]) / (Ts * Ts)
    states = dict(x=x.tolist(), dx=dx.tolist(), ddx=ddx.tolist())
    if shutter_delay:
        tau = np.asarray(tau, np.float64)
        if tau.ndim == 2:      # variable mode: tau (N, C) -> [[tau[n, c] for n] for c] (:553-554)
            states['shutter_delay'] = tau.T.tolist()
        else:                  # const mode: [[tau[c]] * N for c] (:551-552)
            states['shutter_delay'] = [[float(t)] * N for t in tau]
    return states


def solve(meas, w, camera_params, mode, fps, X0, shutter_delay=True, interpolation_mode='vel', tau0=None,
          ctx=None, shutter_delay_mode='const', **opts):
    """Array-level FTE solve. meas (N,C,L,2), w (N,C,L); returns (X (N+2,P), tau, report) with
    tau (C,) for shutter_delay_mode 'const' and (N, C) for 'variable'."""
    k_arr, d_arr, r_arr, t_arr = camera_params[:4]
    n = len(k_arr)
    cams = _native.pack_cameras(k_arr, np.asarray(d_arr).reshape(n, 4), r_arr, np.asarray(t_arr).reshape(n, 3))
    ctx = ctx or _native.default_context()
    o = ctx.fte_default_opts(**opts)
    im = INTERMODES[interpolation_mode] if shutter_delay else 0
    return ctx.fte_solve(build_table(mode), cams, meas, w, 1.0 / float(fps), model_weights(mode), X0, tau0,
                         shutter_delay=shutter_delay, intermode=im, opts=o, sd_mode=shutter_delay_mode)


def fte(OUT_DIR, points_2d_df, mode, camera_params, start_frame, end_frame, dlc_thresh, scene_fpath,
        params: Dict = {}, shutter_delay: bool = False, shutter_delay_mode: str = 'const',
        interpolation_mode: str = 'pos', video: bool = True, plot: bool = False, **solver_opts) -> str:
    sd, sd_mode, intermode = shutter_delay, shutter_delay_mode, interpolation_mode
    if sd:
        assert sd_mode == 'const' or sd_mode == 'variable'
        assert intermode == 'vel' or intermode == 'acc'
    else:
        assert intermode == 'pos'
    os.makedirs(OUT_DIR, exist_ok=True)
    app.start_logging(os.path.join(OUT_DIR, 'fte.log'))
    try:
        t0 = time()
        k_arr, d_arr, r_arr, t_arr, cam_res, n_cams = camera_params
        d_arr = np.asarray(d_arr).reshape((-1, 4))
        markers = get_markers(mode)
        params = dict(params)
        params.update(start_frame=start_frame, end_frame=end_frame, dlc_thresh=dlc_thresh, redesc_a=REDESC_A,
                      redesc_b=REDESC_B, redesc_c=REDESC_C, scene_fpath=scene_fpath, R=R_MEAS,
                      Q={k: Q_TABLE[k] for k in get_pose_params(mode)})
        with open(os.path.join(OUT_DIR, 'reconstruction_params.json'), 'w') as f:
            json.dump(params, f)
        print('----- Generating pairwise 3D points -----')
        points_3d_df = utils.get_pairwise_3d_points_from_df(points_2d_df.query(f'likelihood > {dlc_thresh}'),
                                                            k_arr, d_arr, r_arr, t_arr)
        meas, w = build_measurements(points_2d_df, markers, n_cams, start_frame, end_frame, dlc_thresh)
        X0 = initial_state(points_3d_df, mode, start_frame, end_frame)
        print('\nInitialization took {0:.2f} seconds\n'.format(time() - t0))
        print('----- Optimization (GPU LM) -----')
        t0 = time()
        X, tau, rep = solve(meas, w, (k_arr, d_arr, r_arr, t_arr), mode, params['vid_fps'], X0, sd, intermode,
                            shutter_delay_mode=sd_mode, **solver_opts)
        print(f"status {rep['status_name']}, {rep['iters']} iterations, cost {rep['cost_before']:.6e} -> "
              f"{rep['cost_after']:.6e}")
        print('\nOptimization took {0:.2f} seconds\n'.format(time() - t0))
    finally:
        app.stop_logging()
    N = end_frame - start_frame + 1
    states = states_from_solution(X, tau, 1.0 / float(params['vid_fps']), sd, N)
    positions_3ds = misc.get_all_marker_coords_from_states(states, n_cams, mode=mode, directions=True,
                                                           intermode=intermode)
    import pandas as pd
    frames = np.arange(start_frame, end_frame + 1)
    points_3d_dfs = []
    for pos in positions_3ds:
        points_3d_dfs.append(pd.DataFrame({
            'frame': np.repeat(frames[None, :], len(markers), 0).ravel().astype(np.int64),
            'marker': np.repeat(np.array(markers, dtype=object), N),
            'x': pos[:, :len(markers), 0].T.ravel(), 'y': pos[:, :len(markers), 1].T.ravel(),
            'z': pos[:, :len(markers), 2].T.ravel()}))
    pix_errors = metric.residual_error(points_2d_df, points_3d_dfs, markers, camera_params)
    states['reprj_errors'] = pix_errors
    # fte.pickle keeps the reference's schema (src/core/fte.py:540-579); the LM report (status,
    # iterations, costs) goes beside it
    with open(os.path.join(OUT_DIR, 'solver_report.json'), 'w') as f:
        json.dump({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in rep.items()}, f,
                  default=lambda o: o.item() if hasattr(o, 'item') else str(o))
    return app.save_fte(states, mode, OUT_DIR, scene_fpath, start_frame, directions=True, intermode=intermode,
                        save_videos=video)
