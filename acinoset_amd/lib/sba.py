"""Mirror of src/lib/sba.py (points-only SBA and its data glue) on the GPU.

* `bundle_adjust_points_only` (:181-195) -> acs_sba_points: the same robust objective
  (Cauchy, f_scale, residual = reprojection - observation) minimised per point by the
  fused LM kernel; returns (obj_pts, {'before', 'after'}) exactly like the reference.
* `cost_func_points_only` (:149-153) -> acs_sba_residuals.
* `_sba_points` (:285-313) keeps the reference's point selection (adjacent-pair
  triangulation + inner merge on (frame, marker)) and index semantics.
* `bundle_adjust_points_and_extrinsics` (:158-178) -> acs_sba_extrinsics (Schur LM).
* Calibration-board front end (:37-137, :196-282): `prepare_calib_board_data_for_bundle_
  adjustment`, `prepare_manual_points_for_bundle_adjustment`, `bundle_adjust_board_points_only`
  and `_sba_board_points`, with every image's first-two-camera triangulation batched into one
  GPU call (acs_triangulate_pairs) and the joint points + extrinsics solve on the GPU.
"""
from time import time

import numpy as np

from .. import _native
from .utils import get_pairwise_3d_points_from_df, load_manual_points, load_points, load_scene, save_scene


def create_bundle_adjustment_jacobian_sparsity_matrix(n_cams, n_params_per_camera, camera_indices, n_points,
                                                      point_indices):
    """The Jacobian sparsity pattern of `src/lib/sba.py:11-22` as metadata (the GPU solver
    works on the per-point blocks directly and never builds it): residual rows 2i, 2i+1 of
    observation i touch its camera's parameter columns and its point's 3 columns, laid
    out [cameras | points]. Built in one COO pass and returned as a lil matrix of ints."""
    from scipy.sparse import coo_matrix
    cam = np.asarray(camera_indices, np.int64)
    pt = np.asarray(point_indices, np.int64)
    n_obs = cam.size
    cols_per_obs = np.concatenate([cam[:, None] * n_params_per_camera + np.arange(n_params_per_camera),
                                   n_cams * n_params_per_camera + pt[:, None] * 3 + np.arange(3)], 1)
    k = cols_per_obs.shape[1]
    rows = (2 * np.arange(n_obs)[:, None, None] + np.arange(2)[None, :, None]).repeat(k, 2)
    cols = np.broadcast_to(cols_per_obs[:, None, :], rows.shape)
    shape = (2 * n_obs, n_cams * n_params_per_camera + 3 * n_points)
    A = coo_matrix((np.ones(rows.size, int), (rows.ravel(), cols.ravel())), shape=shape).tolil()
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


# ---- calibration-board front end (src/lib/sba.py:37-137, :196-282) -----------------------

def _triangulate_batch(jobs, k_arr, d_arr, r_arr, t_arr, triangulate_func):
    """jobs: [(uv_a (n,2), uv_b (n,2), cam_a, cam_b)] -> list of (n, 3). The fisheye model
    (triangulate_func None or calib.triangulate_points_fisheye) runs as ONE GPU batch;
    any other triangulate_func is called per job, as the reference does."""
    from .calib import triangulate_points_fisheye
    if not jobs:
        return []
    if triangulate_func is not None and triangulate_func is not triangulate_points_fisheye:
        return [np.asarray(triangulate_func(a, b, k_arr[ca], d_arr[ca], r_arr[ca], t_arr[ca],
                                            k_arr[cb], d_arr[cb], r_arr[cb], t_arr[cb])).reshape(-1, 3)
                for a, b, ca, cb in jobs]
    cams = _native.pack_cameras(k_arr, np.asarray(d_arr).reshape(-1, 4), r_arr, t_arr)
    uva = np.concatenate([np.asarray(a, np.float64).reshape(-1, 2) for a, _, _, _ in jobs])
    uvb = np.concatenate([np.asarray(b, np.float64).reshape(-1, 2) for _, b, _, _ in jobs])
    cia = np.concatenate([np.full(len(np.asarray(a).reshape(-1, 2)), ca, np.int32) for a, _, ca, _ in jobs])
    cib = np.concatenate([np.full(len(np.asarray(a).reshape(-1, 2)), cb, np.int32) for a, _, _, cb in jobs])
    xyz = _native.default_context().triangulate_pairs(cams, uva, uvb, cia, cib)
    out, o = [], 0
    for a, _, _, _ in jobs:
        n = len(np.asarray(a).reshape(-1, 2))
        out.append(xyz[o:o + n])
        o += n
    return out


def prepare_calib_board_data_for_bundle_adjustment(img_pts_arr, fnames_arr, board_shape, k_arr, d_arr, r_arr,
                                                   t_arr, triangulate_func=None):
    """`src/lib/sba.py:37-92`: every image name seen by at least two cameras contributes its
    board corners once per camera that saw it (u,v), one 3-D point per corner, initialised
    by triangulating the first two of those cameras. Returns (points_2d (n_obs,2) float32,
    points_3d (n_pts,3) float32, point_3d_indices, camera_indices).

    The reference walks the image names in the iteration order of a Python `set` of
    strings, which depends on PYTHONHASHSEED; here the order is sorted, so it is
    reproducible. Any order gives the same problem up to a permutation of the points."""
    n_cam = len(img_pts_arr)
    lists = [list(f) for f in fnames_arr]
    seen = {}
    for fnames in lists:
        for fn in set(fnames):
            seen[fn] = seen.get(fn, 0) + 1
    ppi = board_shape[0] * board_shape[1]
    points_2d, point_3d_indices, camera_indices, jobs = [], [], [], []
    counter = 0
    for fn in sorted(k for k, v in seen.items() if v >= 2):
        tri = []
        for cam in range(n_cam):
            if fn in lists[cam]:
                f_idx = lists[cam].index(fn)
                tri.append((cam, f_idx))
                points_2d.append(np.asarray(img_pts_arr[cam][f_idx]).reshape(ppi, 2))
                point_3d_indices.append(np.arange(counter, counter + ppi))
                camera_indices.append(np.full(ppi, cam))
        (a, a_pt), (b, b_pt) = tri[0], tri[1]
        jobs.append((img_pts_arr[a][a_pt], img_pts_arr[b][b_pt], a, b))
        counter += ppi
    points_3d = _triangulate_batch(jobs, k_arr, d_arr, r_arr, t_arr, triangulate_func)
    if not jobs:
        return (np.zeros((0, 2), np.float32), np.zeros((0, 3), np.float32), np.zeros(0, np.int64),
                np.zeros(0, np.int64))
    return (np.concatenate(points_2d).astype(np.float32), np.concatenate(points_3d).astype(np.float32),
            np.concatenate(point_3d_indices).astype(np.int64), np.concatenate(camera_indices).astype(np.int64))


def prepare_manual_points_for_bundle_adjustment(img_pts_arr, k_arr, d_arr, r_arr, t_arr, triangulate_func=None):
    """`src/lib/sba.py:95-137`: img_pts_arr (n_points, n_cams, 2) with NaN where a camera did
    not label the point; a point seen by >= 2 cameras becomes one 3-D point initialised
    from its first two cameras. Returns the four arrays of the board variant."""
    pts = np.asarray(img_pts_arr).swapaxes(0, 1)  # (n_cams, n_points, 2)
    n_cam, n_pts = pts.shape[0], pts.shape[1]
    points_2d, point_3d_indices, camera_indices, jobs = [], [], [], []
    idx = 0
    for i in range(n_pts):
        cams = [c for c in range(n_cam) if not np.isnan(pts[c, i]).any()]
        if len(cams) > 1:
            points_2d.extend(pts[c, i] for c in cams)
            camera_indices.extend(cams)
            point_3d_indices.extend([idx] * len(cams))
            jobs.append((pts[cams[0], i], pts[cams[1], i], cams[0], cams[1]))
            idx += 1
    points_3d = _triangulate_batch(jobs, k_arr, d_arr, r_arr, t_arr, triangulate_func)
    return (np.array(points_2d, np.float32).reshape(-1, 2),
            (np.concatenate(points_3d) if points_3d else np.zeros((0, 3))).astype(np.float32),
            np.array(point_3d_indices, np.int64), np.array(camera_indices, np.int64))


def bundle_adjust_board_points_only(img_pts_arr, fnames_arr, board_shape, k_arr, d_arr, r_arr, t_arr,
                                    triangulate_func=None, project_func=None):
    """`src/lib/sba.py:196-204`."""
    p2, p3, pi, ci = prepare_calib_board_data_for_bundle_adjustment(img_pts_arr, fnames_arr, board_shape, k_arr,
                                                                    d_arr, r_arr, t_arr, triangulate_func)
    return bundle_adjust_points_only(p2, p3, pi, ci, k_arr, d_arr, r_arr, t_arr, project_func)


def _sba_board_points(scene_fpath, points_fpaths, manual_points_fpath, out_fpath, triangulate_func=None,
                      project_func=None, camera_indices=None, manual_points_only=False):
    """`src/lib/sba.py:209-282`: board corners (+ optional hand-labelled points) -> joint
    points + extrinsics SBA -> refined scene JSON at out_fpath. Returns the residuals.

    Kept as the reference has it: manual point indices are offset by the LAST board point
    index (`manual + board.max()`, :249), so the first manual point shares its index with
    the last board corner and the final initial 3-D point is unused."""
    img_pts_arr, fnames_arr, board_shape = [], [], None
    if camera_indices is None:
        camera_indices = range(len(points_fpaths))
    for i in camera_indices:
        points, fnames, board_shape, *_ = load_points(points_fpaths[i])
        img_pts_arr.append(points)
        fnames_arr.append(fnames)
    k_arr, d_arr, r_arr, t_arr, cam_res = load_scene(scene_fpath)
    assert len(k_arr) == len(img_pts_arr)
    if manual_points_fpath is not None:
        manual_points, _, *_ = load_manual_points(manual_points_fpath)
        m2, m3, mi, mc = prepare_manual_points_for_bundle_adjustment(manual_points, k_arr, d_arr, r_arr, t_arr,
                                                                     triangulate_func)
        if manual_points_only:
            print('bundle_adjust_board_points_and_extrinsics (with manual points only)')
            p2, p3, pi, ci = m2, m3, mi, mc
        else:
            print('bundle_adjust_board_points_and_extrinsics (with manual points)')
            p2, p3, pi, ci = prepare_calib_board_data_for_bundle_adjustment(img_pts_arr, fnames_arr, board_shape,
                                                                            k_arr, d_arr, r_arr, t_arr,
                                                                            triangulate_func)
            p2 = np.append(p2, m2, axis=0)
            p3 = np.append(p3, m3, axis=0)
            pi = np.append(pi, mi + pi.max(), axis=0)
            ci = np.append(ci, mc, axis=0)
    else:
        print('bundle_adjust_board_points_and_extrinsics')
        p2, p3, pi, ci = prepare_calib_board_data_for_bundle_adjustment(img_pts_arr, fnames_arr, board_shape, k_arr,
                                                                        d_arr, r_arr, t_arr, triangulate_func)
    obj_pts, r_arr, t_arr, res = bundle_adjust_points_and_extrinsics(p2, p3, pi, ci, k_arr, d_arr, r_arr, t_arr,
                                                                     project_func)
    print(f"\nBefore: mean: {np.mean(res['before'])}, std: {np.std(res['before'])}")
    print(f"After: mean: {np.mean(res['after'])}, std: {np.std(res['after'])}\n")
    save_scene(out_fpath, k_arr, d_arr, r_arr, t_arr, cam_res)
    return res
