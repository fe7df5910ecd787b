"""Mirror of the fisheye part of src/lib/calib.py used by the SBA / FTE path.

project_points_fisheye (:132-136) and triangulate_points_fisheye (:120-129) run on the
GPU (acs_project_fisheye, acs_triangulate_pairs). The board-point bundle adjustment that
refines a calibrated scene is in `lib.sba._sba_board_points` / `lib.app.sba_board_points_
fisheye`; OpenCV's checkerboard detection and per-camera / stereo calibration
(:141-297) stay out of scope (one-off, OpenCV-bound).
"""
import numpy as np

from .. import _native


def _cam(k, d, r, t):
    return _native.pack_cameras(np.asarray(k).reshape(1, 3, 3), np.asarray(d).reshape(1, 4),
                                np.asarray(r).reshape(1, 3, 3), np.asarray(t).reshape(1, 3))


def project_points_fisheye(obj_pts, k, d, r, t, shutter_delay_param=None):
    """(n, 3) world points -> (n, 2) pixels for one camera (R as a 3x3 matrix)."""
    pts = np.asarray(obj_pts, np.float64).reshape(-1, 3)
    return _native.default_context().project(_cam(k, d, r, t), pts)


def triangulate_points_fisheye(img_pts_1, img_pts_2, k1, d1, r1, t1, k2, d2, r2, t2):
    """Two-view fisheye triangulation -> (n, 3)."""
    a = np.asarray(img_pts_1, np.float64).reshape(-1, 2)
    b = np.asarray(img_pts_2, np.float64).reshape(-1, 2)
    cams = np.concatenate([_cam(k1, d1, r1, t1), _cam(k2, d2, r2, t2)])
    return _native.default_context().triangulate_pairs(cams, a, b, 0, 1)
