"""`core.tri` (src/core/tri.py:27-64): filter by likelihood and frame window, pairwise
fisheye triangulation of adjacent cameras on the GPU (`lib.utils.get_pairwise_3d_points_
from_df` -> `acs_triangulate_pairs`), reprojection table, tri.pickle (+ .mat) and the
cam*_tri reprojections (`lib.app.save_tri`).

The reference's `save_error_dists` (src/core/metrics.py:26-93, PDF histograms) is
reporting, out of scope; the error tables it would plot are kept
in tri.pickle as the reference keeps them."""
import json
import os
from typing import Dict

import numpy as np

from ..lib import app, metric, misc, utils


def tri(DATA_DIR, points_2d_df, start_frame, end_frame, dlc_thresh, camera_params, scene_fpath,
        params: Dict = {}) -> str:
    OUT_DIR = os.path.join(DATA_DIR, 'tri')
    os.makedirs(OUT_DIR, exist_ok=True)
    markers = misc.get_markers(mode='all')
    k_arr, d_arr, r_arr, t_arr, _, _ = camera_params
    params = dict(params)
    params.update(start_frame=start_frame, end_frame=end_frame, dlc_thresh=dlc_thresh)
    with open(os.path.join(OUT_DIR, 'reconstruction_params.json'), 'w') as f:
        json.dump(params, f)
    points_2d_df = points_2d_df.query(f'likelihood > {dlc_thresh}')
    points_2d_df = points_2d_df[points_2d_df['frame'].between(start_frame, end_frame)]
    points_3d_df = utils.get_pairwise_3d_points_from_df(points_2d_df, k_arr, np.asarray(d_arr).reshape((-1, 4)),
                                                        r_arr, t_arr)
    points_3d_df['point_index'] = points_3d_df.index
    pix_errors = metric.residual_error(points_2d_df, points_3d_df, markers, camera_params)
    positions = np.full((end_frame - start_frame + 1, len(markers), 3), np.nan)
    mi = {m: i for i, m in enumerate(markers)}
    keep = points_3d_df['marker'].isin(mi)
    sel = points_3d_df[keep]
    fr = sel['frame'].to_numpy().astype(int) - start_frame
    mk = np.array([mi[m] for m in sel['marker']], dtype=int)
    positions[fr, mk] = sel[['x', 'y', 'z']].to_numpy(np.float64)
    return app.save_tri(positions, OUT_DIR, scene_fpath, markers, start_frame, pix_errors, save_videos=True)
