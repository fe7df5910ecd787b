"""Oracle: fisheye camera model, undistortion and pairwise triangulation.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* `project`      — `project_points_fisheye` (`src/lib/calib.py:132-136`) = OpenCV
                   `fisheye::projectPoints` with alpha = 0; identical to the
                   reference's own restatement `pt3d_to_2d` (`src/core/fte.py:80-96`)
                   except for OpenCV's `r > 1e-8` guard (FTE uses sqrt(r^2 + 1e-12)).
* `project_jac`  — analytic d(u,v)/dX used by the oracle LM solvers.
* `undistort`    — `cv.fisheye.undistortPoints` (`src/lib/calib.py:123-124`).
* `triangulate_pair` — `triangulate_points_fisheye` (`src/lib/calib.py:120-129`).
* `pairwise_points` — `get_pairwise_3d_points_from_df` (`src/lib/utils.py:319-349`).
"""
import numpy as np


def _cam(K, D, R, t):
    K = np.asarray(K, np.float64)
    return (K[..., 0, 0], K[..., 1, 1], K[..., 0, 2], K[..., 1, 2],
            np.asarray(D, np.float64).reshape(K.shape[:-2] + (4,)),
            np.asarray(R, np.float64), np.asarray(t, np.float64).reshape(K.shape[:-2] + (3,)))


def project(X, K, D, R, t, fte_form=False):
    """X (n,3); K (n,3,3) or (3,3) ... -> (n,2)."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    fx, fy, cx, cy, d, R, t = _cam(K, D, R, t)
    Y = np.einsum('...ij,...j->...i', R, X) + t
    a = Y[..., 0] / Y[..., 2]
    b = Y[..., 1] / Y[..., 2]
    if fte_form:
        r = np.sqrt(a * a + b * b + 1e-12)
    else:
        r = np.sqrt(a * a + b * b)
    th = np.arctan(r)
    th2 = th * th
    thd = th * (1 + th2 * (d[..., 0] + th2 * (d[..., 1] + th2 * (d[..., 2] + th2 * d[..., 3]))))
    if fte_form:
        s = thd / r
    else:
        big = r > 1e-8
        s = np.where(big, thd / np.where(big, r, 1.0), 1.0)
    return np.stack([fx * a * s + cx, fy * b * s + cy], -1)


def project_jac(X, K, D, R, t):
    """Projection and its Jacobian d(u,v)/dX: returns (uv (n,2), J (n,2,3))."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    fx, fy, cx, cy, d, R, t = _cam(K, D, R, t)
    Y = np.einsum('...ij,...j->...i', R, X) + t
    iz = 1.0 / Y[..., 2]
    a = Y[..., 0] * iz
    b = Y[..., 1] * iz
    r2 = a * a + b * b
    r = np.sqrt(r2)
    th = np.arctan(r)
    th2 = th * th
    k1, k2, k3, k4 = d[..., 0], d[..., 1], d[..., 2], d[..., 3]
    poly = 1 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4)))
    thd = th * poly
    dthd = 1 + th2 * (3 * k1 + th2 * (5 * k2 + th2 * (7 * k3 + th2 * 9 * k4)))
    big = r2 > 1e-16
    rs = np.where(big, r, 1.0)
    s = np.where(big, thd / rs, 1.0)
    # s'(r)/r = (thd'(th) * r / (1 + r^2) - thd) / r^3
    sp_r = np.where(big, (dthd * rs / (1 + r2) - thd) / (rs * rs * rs), 0.0)
    u = fx * a * s + cx
    v = fy * b * s + cy
    duda = fx * (s + a * a * sp_r)
    dudb = fx * a * b * sp_r
    dvda = fy * a * b * sp_r
    dvdb = fy * (s + b * b * sp_r)
    # d(a,b)/dY
    J_ab = np.zeros(a.shape + (2, 3))
    J_ab[..., 0, 0] = iz
    J_ab[..., 0, 2] = -a * iz
    J_ab[..., 1, 1] = iz
    J_ab[..., 1, 2] = -b * iz
    J_uv_ab = np.stack([np.stack([duda, dudb], -1), np.stack([dvda, dvdb], -1)], -2)
    J = J_uv_ab @ J_ab @ R
    return np.stack([u, v], -1), J


def undistort(pts, K, D, iters=10, eps=1e-8):
    """cv::fisheye::undistortPoints (no R, no P): normalised coordinates (n,2)."""
    pts = np.asarray(pts, np.float64).reshape(-1, 2)
    K = np.asarray(K, np.float64)
    k = np.asarray(D, np.float64).ravel()
    pw = (pts - [K[0, 2], K[1, 2]]) / [K[0, 0], K[1, 1]]
    theta_d = np.clip(np.hypot(pw[:, 0], pw[:, 1]), -np.pi / 2, np.pi / 2)
    theta = theta_d.copy()
    active = np.abs(theta_d) > 1e-8
    converged = ~active
    for _ in range(iters):
        t2 = theta * theta
        t4 = t2 * t2
        t6 = t4 * t2
        t8 = t6 * t2
        fix = (theta * (1 + k[0] * t2 + k[1] * t4 + k[2] * t6 + k[3] * t8) - theta_d) / \
              (1 + 3 * k[0] * t2 + 5 * k[1] * t4 + 7 * k[2] * t6 + 9 * k[3] * t8)
        upd = active & ~converged
        theta = np.where(upd, theta - fix, theta)
        converged = converged | (upd & (np.abs(fix) < eps))
    scale = np.where(active, np.tan(theta) / np.where(active, theta_d, 1.0), 1.0)
    flipped = ((theta_d < 0) & (theta > 0)) | ((theta_d > 0) & (theta < 0))
    out = pw * np.where(active, scale, 0.0)[:, None]
    bad = ~converged | flipped
    out[bad] = -1e6
    return out


def triangulate_pair(pa, pb, Ka, Da, Ra, ta, Kb, Db, Rb, tb):
    """Undistort both views, then homogeneous DLT (last right-singular vector)."""
    xa = undistort(pa, Ka, Da)
    xb = undistort(pb, Kb, Db)
    Pa = np.hstack([np.asarray(Ra), np.asarray(ta).reshape(3, 1)])
    Pb = np.hstack([np.asarray(Rb), np.asarray(tb).reshape(3, 1)])
    A = np.stack([xa[:, 0:1] * Pa[2] - Pa[0], xa[:, 1:2] * Pa[2] - Pa[1],
                  xb[:, 0:1] * Pb[2] - Pb[0], xb[:, 1:2] * Pb[2] - Pb[1]], axis=1)
    _, _, Vt = np.linalg.svd(A)
    Xh = Vt[:, -1, :]
    return Xh[:, :3] / Xh[:, 3:4]


def pairwise_points(frame, camera, marker, x, y, K, D, R, t):
    """`get_pairwise_3d_points_from_df` on flat arrays: adjacent pairs (i, i+1 mod C),
    inner join on (frame, marker), triangulate, mean over pairs per (frame, marker).
    Returns (frames, markers, xyz) sorted by (frame, marker)."""
    C = len(K)
    acc = {}
    for ca in range(C):
        cb = (ca + 1) % C
        ia = np.nonzero(camera == ca)[0]
        ib = np.nonzero(camera == cb)[0]
        kb = {(frame[i], marker[i]): i for i in ib}
        pairs = [(i, kb[(frame[i], marker[i])]) for i in ia if (frame[i], marker[i]) in kb]
        if not pairs:
            continue
        ia2 = np.array([p[0] for p in pairs])
        ib2 = np.array([p[1] for p in pairs])
        X = triangulate_pair(np.stack([x[ia2], y[ia2]], -1), np.stack([x[ib2], y[ib2]], -1),
                             K[ca], D[ca], R[ca], t[ca], K[cb], D[cb], R[cb], t[cb])
        for j, i in enumerate(ia2):
            acc.setdefault((frame[i], marker[i]), []).append(X[j])
    keys = sorted(acc)
    xyz = np.array([np.mean(acc[k], axis=0) for k in keys]) if keys else np.zeros((0, 3))
    return (np.array([k[0] for k in keys], np.int64), np.array([k[1] for k in keys], np.int64), xyz)
