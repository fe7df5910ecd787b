"""Mirror of the SBA / FTE seams of src/lib/app.py: `sba_points_fisheye` (:135-138),
`sba_board_points_fisheye` (:123-126), `save_tri` (:238-268), `save_sba` (:271-295),
`save_ekf` (:298-314), `save_fte` (:317-332), `start_logging` / `stop_logging` (:337-345).
The save functions write the pickle/.mat outputs and, when `cam[1-9].mp4` sit beside the
output directory, the per-camera 2-D reprojections (`utils.save_3d_cheetah_as_2d`, GPU
projection). Labelled-video rendering (OpenCV / multiprocessing) is out of scope
(DESIGN.md §7): `save_videos` is accepted and ignored."""
import os
import sys
from glob import glob

import numpy as np

from . import misc, utils
from .calib import project_points_fisheye, triangulate_points_fisheye
from .sba import _sba_board_points, _sba_points


def sba_points_fisheye(scene_fpath, points_2d_df):
    return _sba_points(scene_fpath, points_2d_df, triangulate_points_fisheye, project_points_fisheye)


def sba_board_points_fisheye(scene_fpath, points_fpaths, out_fpath, manual_points_fpath=None, manual_points_only=False,
                             camera_indices=None):
    return _sba_board_points(scene_fpath, points_fpaths, manual_points_fpath, out_fpath, triangulate_points_fisheye,
                             project_points_fisheye, camera_indices, manual_points_only)


def _gaze_targets(head_pos, nose_pos, r_eye_pos, r=3.0):
    """`get_gaze_target_from_positions` (src/lib/misc.py:107-119), vectorised."""
    from scipy.spatial.transform import Rotation
    out = []
    for h, n, e in zip(head_pos, nose_pos, r_eye_pos):
        vn = (n - h) / np.linalg.norm(n - h)
        ve = (e - h) / np.linalg.norm(e - h)
        out.append(h + r * Rotation.from_mrp(np.tan(np.pi / 4 / 4) * ve).apply(vn))
    return np.array(out)


def _videos(out_dir):
    """The original videos, in the parent of the output directory (`src/lib/app.py:239`)."""
    return sorted(glob(os.path.join(os.path.dirname(out_dir), 'cam[1-9].mp4')))


def _with_directions(positions, markers):
    """Append the centre of the eyes ('coe') and the gaze target as two more markers
    (`src/lib/app.py:242-251`); `markers` is extended in place as the reference does."""
    nose, r_eye, l_eye = positions[:, 0, :], positions[:, 1, :], positions[:, 2, :]
    head = np.mean([r_eye, l_eye], axis=0)
    with np.errstate(invalid='ignore'):
        gaze = _gaze_targets(head, nose, r_eye)
    markers += ['coe', 'gaze_target']
    return np.concatenate((positions, head[:, None], gaze[:, None]), axis=1)


def save_tri(positions, out_dir, scene_fpath, markers, start_frame, errors, save_videos=True) -> str:
    """`src/lib/app.py:238-268`: tri.pickle = {positions (N, L+2, 3), start_frame, errors}
    (+ tri.mat without the error tables) and the cam*_tri reprojections."""
    n_vid = len(_videos(out_dir))
    positions = _with_directions(positions, markers)
    out_fpath = os.path.join(out_dir, 'tri.pickle')
    utils.save_optimised_cheetah(positions, out_fpath, extra_data=dict(start_frame=start_frame, errors=errors))
    utils.save_3d_cheetah_as_2d([positions] * n_vid, out_dir, scene_fpath, markers, project_points_fisheye,
                                start_frame)
    return out_fpath


def save_sba(positions, out_dir, scene_fpath, markers, start_frame, save_videos=True) -> str:
    """`src/lib/app.py:271-295`: sba.pickle (+ .mat) and the cam*_sba reprojections."""
    n_vid = len(_videos(out_dir))
    positions = _with_directions(positions, markers)
    out_fpath = os.path.join(out_dir, 'sba.pickle')
    utils.save_optimised_cheetah(positions, out_fpath, extra_data=dict(start_frame=start_frame))
    utils.save_3d_cheetah_as_2d([positions] * n_vid, out_dir, scene_fpath, markers, project_points_fisheye,
                                start_frame)
    return out_fpath


def save_fte(states, mode, out_dir, scene_fpath, start_frame, intermode='pos', directions=True, save_videos=True,
             n_cam=None) -> str:
    """fte.pickle = {positions: per-camera (N, L+2, 3) list, x, dx, ddx, [shutter_delay], reprj_errors,
    start_frame} (+ fte.mat). The reference sizes `positions` by the number of cam*.mp4
    videos next to out_dir (an empty list without videos); `n_cam` overrides that count."""
    if n_cam is None:
        n_cam = len(_videos(out_dir))
    pos = misc.get_all_marker_coords_from_states(states, n_cam, mode=mode, intermode=intermode,
                                                 directions=directions)
    out_fpath = os.path.join(out_dir, 'fte.pickle')
    utils.save_optimised_cheetah(pos, out_fpath, extra_data=dict(**states, start_frame=start_frame))
    bodyparts = misc.get_markers(mode, directions=directions)
    utils.save_3d_cheetah_as_2d(pos, out_dir, scene_fpath, bodyparts, project_points_fisheye, start_frame)
    return out_fpath


def save_ekf(states, mode, out_dir, scene_fpath, start_frame, directions=True, save_videos=True) -> str:
    """`src/lib/app.py:298-314`: ekf.pickle = {positions (filtered), smoothed_positions,
    x, dx, ddx, smoothed_x, smoothed_dx, smoothed_ddx, start_frame} (+ ekf.mat) and the
    cam*_ekf reprojections of the smoothed positions. Labelled videos are out of scope
    (DESIGN.md §7)."""
    n_vid = len(_videos(out_dir))
    positions = [misc.get_3d_marker_coords({'x': x}, directions=directions, mode=mode) for x in states['x']]
    smoothed = [misc.get_3d_marker_coords({'x': x}, directions=directions, mode=mode) for x in states['smoothed_x']]
    out_fpath = os.path.join(out_dir, 'ekf.pickle')
    utils.save_optimised_cheetah(positions, out_fpath, extra_data=dict(smoothed_positions=smoothed, **states,
                                                                       start_frame=start_frame))
    bodyparts = misc.get_markers(mode, directions=directions)
    utils.save_3d_cheetah_as_2d([smoothed] * n_vid, out_dir, scene_fpath, bodyparts, project_points_fisheye,
                                start_frame)
    return out_fpath


def start_logging(out_fpath):
    sys.stdout = misc.Logger(out_fpath)


def stop_logging():
    if isinstance(sys.stdout, misc.Logger):
        sys.stdout.logfile.close()
        sys.stdout = sys.stdout.terminal
