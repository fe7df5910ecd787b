"""Numpy stand-in for the four OpenCV calls the reference SBA path makes.

Used ONLY by `make_golden.py` (in the build container) to run the reference's own
`lib.sba` / `lib.calib` / `lib.utils` / `lib.metric` code, because `cv2` is not
installed. It restates the published OpenCV algorithms:

* `cv::Rodrigues` (rotation vector <-> matrix; matrix input re-orthogonalised by SVD);
* `cv::fisheye::projectPoints` (Kannala-Brandt, alpha = 0, `r > 1e-8` guard);
* `cv::fisheye::undistortPoints` (Newton on theta, default criteria 10 iterations / 1e-8);
* `cv::triangulatePoints` (homogeneous DLT, last right-singular vector).

`nptyping.Array` is stubbed, and `np.float` / `np.int` are re-aliased because the
reference uses them (`src/lib/utils.py:331`, `src/lib/sba.py:90`).
"""
import sys
import types

import numpy as np


def _rodrigues(src):
    src = np.asarray(src, np.float64)
    if src.size == 3:
        r = src.reshape(3)
        th = np.linalg.norm(r)
        if th < np.finfo(np.float64).eps:
            return np.eye(3), None
        k = r / th
        c, s = np.cos(th), np.sin(th)
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        R = c * np.eye(3) + (1 - c) * np.outer(k, k) + s * Kx
        return R, None
    R = src.reshape(3, 3)
    U, _, Vt = np.linalg.svd(R)
    R = U @ Vt
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = np.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = np.clip((np.trace(R) - 1) * 0.5, -1.0, 1.0)
    th = np.arccos(c)
    if s < 1e-5:
        if c > 0:
            r = np.zeros(3)
        else:
            t = (R[0, 0] + 1) * 0.5
            rx = np.sqrt(max(t, 0.0))
            t = (R[1, 1] + 1) * 0.5
            ry = np.sqrt(max(t, 0.0)) * (-1.0 if R[0, 1] < 0 else 1.0)
            t = (R[2, 2] + 1) * 0.5
            rz = np.sqrt(max(t, 0.0)) * (-1.0 if R[0, 2] < 0 else 1.0)
            if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1, 2] > 0) != (ry * rz > 0):
                rz = -rz
            r = np.array([rx, ry, rz])
            r = r * (th / np.linalg.norm(r))
    else:
        r = np.array([rx, ry, rz]) * (th / (2 * s))
    return r.reshape(3, 1), None


def _fisheye_project(obj, rvec, tvec, K, D, alpha=0.0):
    obj = np.asarray(obj, np.float64).reshape(-1, 3)
    R, _ = _rodrigues(rvec)
    t = np.asarray(tvec, np.float64).reshape(3)
    K = np.asarray(K, np.float64)
    k = np.asarray(D, np.float64).ravel()
    Y = obj @ R.T + t
    a = Y[:, 0] / Y[:, 2]
    b = Y[:, 1] / Y[:, 2]
    r = np.sqrt(a * a + b * b)
    th = np.arctan(r)
    th2 = th * th
    th4 = th2 * th2
    thd = th * (1 + k[0] * th2 + k[1] * th4 + k[2] * th4 * th2 + k[3] * th4 * th4)
    big = r > 1e-8
    inv_r = np.where(big, 1.0 / np.where(big, r, 1.0), 1.0)
    cdist = np.where(big, thd * inv_r, 1.0)
    xd0 = a * cdist
    xd1 = b * cdist
    u = K[0, 0] * (xd0 + alpha * xd1) + K[0, 2]
    v = K[1, 1] * xd1 + K[1, 2]
    return np.stack([u, v], -1).reshape(-1, 1, 2), None


def _fisheye_undistort(distorted, K, D, R=None, P=None):
    pts = np.asarray(distorted, np.float64).reshape(-1, 2)
    K = np.asarray(K, np.float64)
    k = np.asarray(D, np.float64).ravel()
    f = np.array([K[0, 0], K[1, 1]])
    c = np.array([K[0, 2], K[1, 2]])
    RR = np.eye(3) if R is None else np.asarray(R, np.float64).reshape(3, 3)
    if P is not None:
        PP = np.asarray(P, np.float64)[:3, :3]
        RR = PP @ RR
    out = np.empty_like(pts)
    for i, pi in enumerate(pts):
        pw = (pi - c) / f
        theta_d = np.sqrt(pw[0] ** 2 + pw[1] ** 2)
        theta_d = min(max(-np.pi / 2, theta_d), np.pi / 2)
        converged = False
        theta = theta_d
        scale = 0.0
        if abs(theta_d) > 1e-8:
            for _ in range(10):
                t2 = theta * theta
                t4 = t2 * t2
                t6 = t4 * t2
                t8 = t6 * t2
                k0t2, k1t4, k2t6, k3t8 = k[0] * t2, k[1] * t4, k[2] * t6, k[3] * t8
                fix = (theta * (1 + k0t2 + k1t4 + k2t6 + k3t8) - theta_d) / \
                      (1 + 3 * k0t2 + 5 * k1t4 + 7 * k2t6 + 9 * k3t8)
                theta = theta - fix
                if abs(fix) < 1e-8:
                    converged = True
                    break
            scale = np.tan(theta) / theta_d
        else:
            converged = True
        flipped = (theta_d < 0 and theta > 0) or (theta_d > 0 and theta < 0)
        if converged and not flipped:
            pu = pw * scale
            pr = RR @ np.array([pu[0], pu[1], 1.0])
            out[i] = pr[:2] / pr[2]
        else:
            out[i] = -1e6
    return out.reshape(-1, 1, 2)


def _triangulate(P1, P2, x1, x2):
    P1 = np.asarray(P1, np.float64)
    P2 = np.asarray(P2, np.float64)
    x1 = np.asarray(x1, np.float64).reshape(-1, 2)
    x2 = np.asarray(x2, np.float64).reshape(-1, 2)
    out = np.empty((4, len(x1)))
    for i in range(len(x1)):
        A = np.stack([x1[i, 0] * P1[2] - P1[0], x1[i, 1] * P1[2] - P1[1],
                      x2[i, 0] * P2[2] - P2[0], x2[i, 1] * P2[2] - P2[1]])
        _, _, Vt = np.linalg.svd(A)
        out[:, i] = Vt[-1]
    return out


def install():
    cv2 = types.ModuleType('cv2')
    cv2.Rodrigues = _rodrigues
    cv2.triangulatePoints = _triangulate
    fe = types.SimpleNamespace(projectPoints=_fisheye_project, undistortPoints=_fisheye_undistort)
    cv2.fisheye = fe
    sys.modules['cv2'] = cv2
    npt = types.ModuleType('nptyping')

    class _Array:
        def __class_getitem__(cls, item):
            return np.ndarray
    npt.Array = _Array
    sys.modules['nptyping'] = npt
    if not hasattr(np, 'float'):
        np.float = float
    if not hasattr(np, 'int'):
        np.int = int
