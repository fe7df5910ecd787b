"""`core.sba` (src/core/sba.py:27-70): filter by likelihood and frame window, GPU SBA,
reprojection metric, sba.pickle."""
import json
import os
from typing import Dict

import numpy as np

from ..lib import app, metric, misc


def sba(DATA_DIR, points_2d_df, start_frame, end_frame, dlc_thresh, camera_params, scene_fpath, params: Dict = {},
        plot: bool = False) -> str:
    OUT_DIR = os.path.join(DATA_DIR, 'sba')
    os.makedirs(OUT_DIR, exist_ok=True)
    app.start_logging(os.path.join(OUT_DIR, 'sba.log'))
    markers = misc.get_markers()
    params = dict(params)
    params.update(start_frame=start_frame, end_frame=end_frame, dlc_thresh=dlc_thresh)
    with open(os.path.join(OUT_DIR, 'reconstruction_params.json'), 'w') as f:
        json.dump(params, f)
    points_2d_df = points_2d_df.query(f'likelihood > {dlc_thresh}')
    points_2d_df = points_2d_df[points_2d_df['frame'].between(start_frame, end_frame)]
    try:
        points_3d_df, residuals = app.sba_points_fisheye(scene_fpath, points_2d_df)
    finally:
        app.stop_logging()
    pix_errors = metric.residual_error(points_2d_df, points_3d_df, markers, camera_params)
    print(f'reprojection RMS: {metric.reprojection_rms(pix_errors):.4f} px')
    positions = np.full((end_frame - start_frame + 1, len(markers), 3), np.nan)
    mi = {m: i for i, m in enumerate(markers)}
    fr = points_3d_df['frame'].to_numpy().astype(int) - start_frame
    mk = np.array([mi[m] for m in points_3d_df['marker']])
    positions[fr, mk] = points_3d_df[['x', 'y', 'z']].to_numpy()
    return app.save_sba(positions, OUT_DIR, scene_fpath, markers, start_frame)
