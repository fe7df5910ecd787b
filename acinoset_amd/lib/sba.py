"""Mirror of src/lib/sba.py (points-only SBA and its data glue) on the GPU.

* `bundle_adjust_points_only` (:181-195) -> acs_sba_points: the same robust objective
  (Cauchy, f_scale, residual = reprojection - observation) minimised per point by the
  fused LM kernel; returns (obj_pts, {'before', 'after'}) exactly like the reference.
* `cost_func_points_only` (:149-153) -> acs_sba_residuals.
* `_sba_points` (:285-313) keeps the reference's point selection (adjacent-pair
  triangulation + inner merge on (frame, marker)) and index semantics.
* `bundle_adjust_points_and_extrinsics` (:158-178) -> acs_sba_extrinsics (Schur LM).
"""
from time import time

import numpy as np

from .. import _native
from .utils import get_pairwise_3d_points_from_df, load_scene


def create_bundle_adjustment_jacobian_sparsity_matrix(n_cams, n_params_per_camera, camera_indices, n_points,
                                                      point_indices):
    """`src/lib/sba.py:11-22` (sparsity metadata; the GPU solver does not need it)."""
    from scipy.sparse import lil_matrix
    m = camera_indices.size * 2
    n = n_cams * n_params_per_camera + n_points * 3
    A = lil_matrix((m, n), dtype=int)
    i = np.arange(camera_indices.size)
    for s in range(n_params_per_camera):
        A[2 * i, camera_indices * n_params_per_camera + s] = 1
        A[2 * i + 1, camera_indices * n_params_per_camera + s] = 1
    for s in range(3):
        A[2 * i, n_cams * n_params_per_camera + point_indices * 3 + s] = 1
        A[2 * i + 1, n_cams * n_params_per_camera + point_indices * 3 + s] = 1
    return A


def _cams(k_arr, d_arr, r_arr, t_arr):
    n = len(k_arr)
    return _native.pack_cameras(k_arr, np.asarray(d_arr).reshape(n, 4), r_arr, np.asarray(t_arr).reshape(n, 3))


def cost_func_points_only(params, n_points, point_3d_indices, camera_indices, k_arr, d_arr, r_arr, t_arr, points_2d,
                          project_func=None):
    obj = np.asarray(params, np.float64).reshape(n_points, 3)
    return _native.default_context().sba_residuals(_cams(k_arr, d_arr, r_arr, t_arr), points_2d, point_3d_indices,
                                                   camera_indices, obj)


def bundle_adjust_points_only(points_2d, points_3d, point_3d_indices, camera_indices, k_arr, d_arr, r_arr, t_arr,
                              project_func=None, f_scale=50, **opts):
    """Points-only robust BA. `project_func` is accepted for signature compatibility: the
    fisheye model is built into the kernel (src/lib/app.py:135-138 passes
    project_points_fisheye)."""
    ctx = _native.default_context()
    o = ctx.sba_opts(f_scale=float(f_scale), **opts)
    t0 = time()
    pts, rb, ra, rep = ctx.sba_points(_cams(k_arr, d_arr, r_arr, t_arr), np.asarray(points_2d, np.float64),
                                      np.asarray(point_3d_indices), np.asarray(camera_indices),
                                      np.asarray(points_3d, np.float64), o)
    t1 = time()
    print(f'GPU SBA: {rep["n_problems"]} points, iters max {rep["iters_max"]}, cost {rep["cost_before"]:.4e} -> '
          f'{rep["cost_after"]:.4e}, status {rep["status_counts"]}')
    print(f'\nOptimization took {t1 - t0:.2f} seconds')
    return pts, dict(before=rb, after=ra)


def _sba_points(scene_fpath, points_2d_df, triangulate_func=None, project_func=None):
    """`src/lib/sba.py:285-313`."""
    k_arr, d_arr, r_arr, t_arr, cam_res = load_scene(scene_fpath)
    points_3d_df = get_pairwise_3d_points_from_df(points_2d_df, k_arr, d_arr.reshape((-1, 4)), r_arr, t_arr,
                                                  triangulate_func)
    points_3d_df['point_index'] = points_3d_df.index
    points_3d = np.array(points_3d_df[['x', 'y', 'z']], dtype=np.float64)
    points_df = points_2d_df.merge(points_3d_df, how='inner', on=['frame', 'marker'], suffixes=('_cam', ''))
    points_2d = np.array(points_df[['x_cam', 'y_cam']], dtype=np.float64)
    point_indices = np.array(points_df['point_index'])
    camera_indices = np.array(points_df['camera'])
    print('bundle_adjust_points_only')
    pts_3d, res = bundle_adjust_points_only(points_2d, points_3d, point_indices, camera_indices, k_arr, d_arr, r_arr,
                                            t_arr, project_func, f_scale=50)
    print(f"\nBefore: mean: {np.mean(res['before'])}, std: {np.std(res['before'])}")
    print(f"After: mean: {np.mean(res['after'])}, std: {np.std(res['after'])}\n")
    new_points_3d_df = points_3d_df.copy()
    new_points_3d_df[['x', 'y', 'z']] = pts_3d
    return new_points_3d_df, res


def rodrigues_to_matrix(rvecs):
    """Rotation vectors (n,3) -> matrices (n,3,3) (cv::Rodrigues, vector -> matrix)."""
    rv = np.asarray(rvecs, np.float64).reshape(-1, 3)
    out = np.empty((len(rv), 3, 3))
    for i, r in enumerate(rv):
        th = np.linalg.norm(r)
        if th < np.finfo(np.float64).eps:
            out[i] = np.eye(3)
            continue
        k = r / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        out[i] = np.cos(th) * np.eye(3) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * Kx
    return out


def matrix_to_rodrigues(R_arr):
    """Rotation matrices (n,3,3) -> rotation vectors (n,3) (cv::Rodrigues, matrix -> vector)."""
    out = []
    for R in np.asarray(R_arr, np.float64).reshape(-1, 3, 3):
        U, _, Vt = np.linalg.svd(R)
        R = U @ Vt
        c = np.clip((np.trace(R) - 1) * 0.5, -1.0, 1.0)
        th = np.arccos(c)
        v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
        s = np.linalg.norm(v) * 0.5
        if s < 1e-5:
            if c > 0:
                out.append(np.zeros(3))
                continue
            w, V = np.linalg.eigh((R + np.eye(3)) * 0.5)
            ax = V[:, np.argmax(w)]
            out.append(ax * th)
            continue
        out.append(v * (th / (2 * s)))
    return np.array(out)


def params_to_points_extrinsics(params, n_cams, n_points):
    """`src/lib/sba.py:25-32`."""
    r_end = n_cams * 3
    t_end = r_end + n_cams * 3
    r_arr = rodrigues_to_matrix(params[:r_end].reshape(n_cams, 3))
    t_arr = params[r_end:t_end].reshape((n_cams, 3, 1))
    obj_pts = params[t_end:].reshape((n_points, 3))
    return obj_pts, r_arr, t_arr


def cost_func_points_extrinsics(params, n_cams, n_points, point_3d_indices, camera_indices, k_arr, d_arr, points_2d,
                                project_func=None):
    """`src/lib/sba.py:142-146`."""
    obj, r_arr, t_arr = params_to_points_extrinsics(np.asarray(params, np.float64), n_cams, n_points)
    return cost_func_points_only(obj.ravel(), n_points, point_3d_indices, camera_indices, k_arr, d_arr, r_arr, t_arr,
                                 points_2d)


def bundle_adjust_points_and_extrinsics(points_2d, points_3d, point_3d_indices, camera_indices, k_arr, d_arr, r_arr,
                                        t_arr, project_func=None, f_scale=1.0, **opts):
    """`src/lib/sba.py:158-178` -> acs_sba_extrinsics: points and every camera's rotation and
    translation refined together (intrinsics fixed) on the same Cauchy objective (scipy's
    default f_scale = 1). Returns (obj_pts (n,3), r_arr (C,3,3), t_arr (C,3,1),
    {'before', 'after'}) like the reference; rotations stay orthonormal matrices (updated
    on SO(3), which is what the reference's Rodrigues round trip represents)."""
    ctx = _native.default_context()
    n = len(k_arr)
    o = ctx.sba_ext_opts(f_scale=float(f_scale), **opts)
    t0 = time()
    cams, pts, rb, ra, rep = ctx.sba_extrinsics(_cams(k_arr, d_arr, r_arr, t_arr), np.asarray(points_2d, np.float64),
                                                np.asarray(point_3d_indices), np.asarray(camera_indices),
                                                np.asarray(points_3d, np.float64), o)
    t1 = time()
    print(f'GPU SBA (points + extrinsics): {len(pts)} points, {n} cameras, {rep["iters"]} iterations, cost '
          f'{rep["cost_before"]:.6e} -> {rep["cost_after"]:.6e} ({rep["status_name"]})')
    print(f'\nOptimization took {t1 - t0:.2f} seconds')
    r_out = cams[:, 8:17].reshape(n, 3, 3).copy()
    t_out = cams[:, 17:20].reshape(n, 3, 1).copy()
    return pts, r_out, t_out, dict(before=rb, after=ra)
