"""Drop-in for `core.ekf` (src/core/ekf.py:26-347): EKF + RTS smoother on the GPU.

The reference's per-frame Python loop (numerical Jacobian by 30 FK + projection calls per
camera, 2CL x 2CL inverse of S) becomes one `acs_ekf_run` call (acinoset_amd/csrc/ekf.hip):
one workgroup walks the frames of a sequence with the measurement model, the
forward-difference Jacobian and the Kalman update in device memory, then the smoother.

Everything around it is the reference's: the initial state from linear fits of the
pairwise-triangulated nose / lure (:121-157), P0 (:159-186), Q (:188-207), R (:241-253),
the outputs and ekf.pickle (:304-347, lib.app.save_ekf). `ref_numerics=True` (default)
reproduces the reference's float32 state rounding (:79); `False` runs in float64.
"""
import json
import os
from time import time
from typing import Dict

import numpy as np

from .. import _native
from ..kinematics import build_table, get_markers, get_pose_params
from ..lib import app, utils

SIGMA_BOUND = 3                                                                   # src/core/ekf.py:52
CAL_COVS = [0.137, 0.236, 0.176, 0.298, 0.087, 0.116]                            # :210
QB_LIST = [5.0, 5.0, 5.0, 10.0, 10.0, 10.0, 5.0, 5.0, 25.0, 5.0, 50.0, 5.0, 50.0, 25.0, 100.0, 30.0, 140.0, 40.0,
           350.0, 200.0, 350.0, 200.0, 450.0, 400.0, 450.0, 400.0, 5.0, 5.0, 5.0]  # :188-203


def _n_angular(mode):
    return len([k for k in get_pose_params(mode) if 'phi' in k or 'theta' in k or 'psi' in k])


def initial_covariance(mode):
    """P0 (src/core/ekf.py:159-186), including the reference's -0.28 neck-length entry."""
    na = _n_angular(mode)
    ang_pos, ang_vel, ang_acc = np.full(na, (np.pi / 4) ** 2), np.full(na, 9.0), np.full(na, 9.0)
    ang_acc[10:] = 25.0
    lin = lambda v: np.full(3, v)  # noqa: E731
    if mode == 'default':
        d = [lin(9.0), ang_pos[:3], [-0.28], ang_pos[3:], lin(9.0),
             lin(25.0), ang_vel[:3], [0.0], ang_vel[3:], lin(25.0),
             lin(9.0), ang_acc[:3], [0.0], ang_acc[3:], lin(9.0)]
    elif mode == 'head':
        d = [lin(9.0), ang_pos[:3], ang_pos[3:], lin(25.0), ang_vel[:3], ang_vel[3:], lin(9.0), ang_acc[:3],
             ang_acc[3:]]
    else:
        raise ValueError(f"core.ekf supports marker_mode 'default' and 'head' (src/core/ekf.py:176-186), "
                         f'not {mode!r}')
    return np.diag(np.concatenate(d))


def process_covariance(P, sT):
    """Q of the constant-acceleration model (src/core/ekf.py:188-207)."""
    qb = np.diag(QB_LIST[:P]) ** 2
    return np.block([[sT ** 4 / 4 * qb, sT ** 3 / 2 * qb, sT ** 2 / 2 * qb],
                     [sT ** 3 / 2 * qb, sT ** 2 * qb, sT * qb],
                     [sT ** 2 / 2 * qb, sT * qb, qb]])


def ring_cal_covs(n_cams):
    """Calibration covariances for a rig of `n_cams` cameras: the reference's six values
    (src/core/ekf.py:210) for six cameras; for other rigs (the synthetic 12-camera ring of
    configs[4], which has no calibration of its own) camera c takes the reference's value of
    camera c mod 6. The reference itself asserts six cameras (:213)."""
    return [CAL_COVS[c % len(CAL_COVS)] for c in range(n_cams)]


def measurement_std(n_cams, cal_covs=None):
    """Per-camera pixel std of R (src/core/ekf.py:244-248): dlc_cov + 2 cov_c / min(cov).
    The reference hard-codes 6 cameras (:213); other rigs pass their own `cal_covs`."""
    cal_covs = CAL_COVS if cal_covs is None else list(cal_covs)
    assert n_cams == len(cal_covs), (n_cams, len(cal_covs))
    return np.array([2 * c / min(cal_covs) for c in cal_covs])


def dense_observations(points_2d_df, markers, n_cams, n_frames):
    """(n_frames, C, L, 2) pixels and (n_frames, C, L) likelihoods, NaN where the
    DataFrame has no row (the reference's stack/unstack pivot, :103-118)."""
    mi = {m: i for i, m in enumerate(markers)}
    meas = np.full((n_frames, n_cams, len(markers), 2), np.nan)
    lik = np.full((n_frames, n_cams, len(markers)), np.nan)
    df = points_2d_df[points_2d_df['marker'].isin(markers) & points_2d_df['frame'].between(0, n_frames - 1)]
    f = df['frame'].to_numpy().astype(int)
    c = df['camera'].to_numpy().astype(int)
    ok = (c >= 0) & (c < n_cams)
    f, c = f[ok], c[ok]
    m = np.array([mi[v] for v in df['marker'][ok]], dtype=int)
    meas[f, c, m, 0] = df['x'].to_numpy(np.float64)[ok]
    meas[f, c, m, 1] = df['y'].to_numpy(np.float64)[ok]
    lik[f, c, m] = df['likelihood'].to_numpy(np.float64)[ok]
    return meas, lik


def _linfit(fr, v):
    A = np.stack([fr, np.ones_like(fr)], 1)
    return np.linalg.lstsq(A, v, rcond=None)[0]


def initial_state(points_3d_df, mode, start_frame, fps):
    """src/core/ekf.py:121-157 (scipy linregress slope / intercept = least-squares line)."""
    idx = get_pose_params(mode)
    P = len(idx)
    sT = 1.0 / fps
    s = np.zeros(3 * P)
    if 'lure' in get_markers(mode):
        lure = points_3d_df[points_3d_df['marker'] == 'lure'][['frame', 'x', 'y']].to_numpy(np.float64)
        if len(lure) >= 2:
            (sx, ix), (sy, iy) = _linfit(lure[:, 0], lure[:, 1]), _linfit(lure[:, 0], lure[:, 2])
            s[[idx['x_l'], idx['y_l']]] = [start_frame * sx + ix, start_frame * sy + iy]
            s[[P + idx['x_l'], P + idx['y_l']]] = [sx / sT, sy / sT]
        else:
            print('Lure initialisation error: no lure points -> Lure states initialised to zero')
    nose = points_3d_df[points_3d_df['marker'] == 'nose'][['frame', 'x', 'y']].to_numpy(np.float64)
    (sx, ix), (sy, iy) = _linfit(nose[:, 0], nose[:, 1]), _linfit(nose[:, 0], nose[:, 2])
    s[[idx['x_0'], idx['y_0'], idx['psi_0']]] = [start_frame * sx + ix, start_frame * sy + iy, np.arctan2(sy, sx)]
    s[[P + idx['x_0'], P + idx['y_0']]] = [sx / sT, sy / sT]
    return s


def run(meas, likelihood, camera_params, mode, fps, s0, dlc_thresh=0.5, ref_numerics=True, cal_covs=None,
        covariances=False, ctx=None, jacobian='fd'):
    """The filter + smoother on (N, C, L, 2) observations from state s0: returns the
    dict of acinoset_amd._native.Context.ekf_run. `jacobian`: 'fd' = the reference's
    forward-difference H (src/core/ekf.py:81-96), 'analytic' = H from the FK Jacobian
    (float64, so with ref_numerics=False)."""
    ctx = ctx or _native.default_context()
    k_arr, d_arr, r_arr, t_arr, cam_res, n_cams = camera_params
    cams = _native.pack_cameras(k_arr, np.asarray(d_arr).reshape(-1, 4), r_arr, np.asarray(t_arr).reshape(-1, 3))
    table = build_table(mode)
    P = table.P
    sT = 1.0 / fps
    return ctx.ekf_run(table, cams, meas, likelihood, fps, dlc_thresh, float(cam_res[0]),
                       measurement_std(n_cams, cal_covs), process_covariance(P, sT), initial_covariance(mode), s0,
                       ref_numerics=ref_numerics, covariances=covariances, jacobian=jacobian)


def ekf(DATA_DIR, points_2d_df, marker_mode, camera_params, start_frame, end_frame, dlc_thresh, scene_fpath,
        params: Dict = {}, ref_numerics=True, cal_covs=None, jacobian='fd') -> str:
    """`src/core/ekf.py:26` signature and outputs (OUT_DIR/ekf/ekf.pickle). `cal_covs`
    (extension): per-camera calibration covariances; None = the reference's six values,
    or `ring_cal_covs(n_cams)` for a rig that is not six cameras. `jacobian` (extension):
    'analytic' replaces the forward-difference H by the FK Jacobian (needs
    ref_numerics=False)."""
    OUT_DIR = os.path.join(DATA_DIR, 'ekf')
    os.makedirs(OUT_DIR, exist_ok=True)
    app.start_logging(os.path.join(OUT_DIR, 'ekf.log'))
    k_arr, d_arr, r_arr, t_arr, cam_res, n_cams = camera_params
    markers = get_markers(marker_mode)
    P = len(get_pose_params(marker_mode))
    fps = params['vid_fps']
    params = dict(params, marker_mode=marker_mode, start_frame=start_frame, end_frame=end_frame,
                  dlc_thresh=dlc_thresh, sigma_bound=SIGMA_BOUND)
    with open(os.path.join(OUT_DIR, 'reconstruction_params.json'), 'w') as f:
        json.dump(params, f)
    points_3d_df = utils.get_pairwise_3d_points_from_df(points_2d_df, k_arr, np.asarray(d_arr).reshape((-1, 4)),
                                                        r_arr, t_arr)
    s0 = initial_state(points_3d_df, marker_mode, start_frame, fps)
    n_total = int(points_2d_df['frame'].max()) + 1
    meas, lik = dense_observations(points_2d_df, markers, n_cams, max(n_total, end_frame + 1))
    t0 = time()
    if cal_covs is None and n_cams != len(CAL_COVS):
        cal_covs = ring_cal_covs(n_cams)
        print(f'\t{n_cams} cameras: calibration covariances {cal_covs} (reference values by camera mod 6)')
    out = run(meas[start_frame:end_frame + 1], lik[start_frame:end_frame + 1], camera_params, marker_mode, fps, s0,
              dlc_thresh, ref_numerics, cal_covs=cal_covs, jacobian=jacobian)
    opt_time = time() - t0
    app.stop_logging()
    xe, xs = out['x_est'], out['x_smooth']
    states = dict(x=xe[:, :P], dx=xe[:, P:2 * P], ddx=xe[:, 2 * P:],
                  smoothed_x=xs[:, :P], smoothed_dx=xs[:, P:2 * P], smoothed_ddx=xs[:, 2 * P:])
    print(f"\tOutliers ignored: {int(out['outliers'])}")
    print('\tOptimization took {0:.2f} seconds'.format(opt_time))
    return app.save_ekf(states, marker_mode, OUT_DIR, scene_fpath, start_frame, save_videos=False)
