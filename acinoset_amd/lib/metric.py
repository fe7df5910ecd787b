"""Mirror of src/lib/metric.py:36-101 (`residual_error`): per-camera table of
reprojection residuals, with the projection on the GPU. Columns are float-typed
(the reference builds them from a mixed-type np.vstack, so every column became a string
and downstream medians failed — SURVEY.md §5); `camera_distance` keeps the reference's
definition (distance to t, not to the camera centre)."""
from typing import Dict

import numpy as np
import pandas as pd

from . import calib

COLUMNS = ['frame', 'marker', 'camera_distance', 'pixel_residual', 'pck_threshold', 'error_u', 'error_v']


def residual_error(points_2d_df, points_3d_dfs, markers, camera_params) -> Dict:
    k_arr, d_arr, r_arr, t_arr, _, _ = camera_params
    n_cam = len(k_arr)
    if not isinstance(points_3d_dfs, list):
        points_3d_dfs = [points_3d_dfs] * n_cam
    error = {str(i): None for i in range(n_cam)}
    for i in range(n_cam):
        cam2d = points_2d_df[points_2d_df['camera'] == i]
        nose = cam2d[cam2d['marker'] == 'nose'].sort_values(by=['frame'])
        l_eye = cam2d[cam2d['marker'] == 'l_eye'].sort_values(by=['frame'])
        r_eye = cam2d[cam2d['marker'] == 'r_eye'].sort_values(by=['frame'])
        eye = l_eye.combine_first(r_eye).drop_duplicates(subset=['frame'], keep='first')
        valid_range = np.intersect1d(cam2d['frame'].to_numpy(), points_3d_dfs[i]['frame'].to_numpy())
        vf = np.intersect1d(np.intersect1d(eye['frame'].to_numpy(), nose['frame'].to_numpy()), valid_range)
        nose = nose[nose['frame'].isin(vf)]
        eye = eye[eye['frame'].isin(vf)]
        n2e = np.linalg.norm(nose[['x', 'y']].to_numpy() - eye[['x', 'y']].to_numpy(), axis=1)
        n2e_df = pd.DataFrame({'frame': nose['frame'].to_numpy(), 'distance': n2e}).set_index('frame')
        dfs = []
        for m in markers:
            p2 = cam2d[cam2d['marker'] == m]
            p3 = points_3d_dfs[i][points_3d_dfs[i]['marker'] == m]
            p2 = p2[p2[['x', 'y']].notnull().all(axis=1)]
            p3 = p3[p3[['x', 'y', 'z']].notnull().all(axis=1)]
            v = np.intersect1d(p2['frame'].to_numpy(), p3['frame'].to_numpy())
            p2 = p2[p2['frame'].isin(v)].sort_values(by=['frame'])
            p3 = p3[p3['frame'].isin(v)].sort_values(by=['frame'])
            if len(p2) == 0 or len(p3) == 0:
                continue
            pck = n2e_df.reindex(v)['distance'].to_numpy()
            pts2 = p2[['x', 'y']].to_numpy(np.float64)
            pts3 = p3[['x', 'y', 'z']].to_numpy(np.float64)
            prj = calib.project_points_fisheye(pts3, k_arr[i], d_arr[i], r_arr[i], t_arr[i])
            cam_dist = np.sqrt(np.sum((pts3 - np.squeeze(t_arr[i])) ** 2, axis=1))
            err = pts2 - prj
            dfs.append(pd.DataFrame({'frame': p2['frame'].to_numpy(), 'marker': m, 'camera_distance': cam_dist,
                                     'pixel_residual': np.sqrt(np.sum(err ** 2, axis=1)), 'pck_threshold': pck,
                                     'error_u': err[:, 0], 'error_v': err[:, 1]}))
        error[str(i)] = pd.concat(dfs, ignore_index=True) if dfs else pd.DataFrame(columns=COLUMNS)
    return error


def reprojection_rms(errors: Dict) -> float:
    """"reproj-px-RMS": RMS of pixel_residual over every camera's valid observations."""
    v = np.concatenate([e['pixel_residual'].to_numpy(np.float64) for e in errors.values()
                        if e is not None and len(e)] or [np.zeros(0)])
    return float(np.sqrt(np.mean(v ** 2))) if v.size else float('nan')
