"""The BASELINE.json configs as concrete synthetic workloads, shared by
`bench.py` and the parity tests so that both run exactly the same problems.

* configs[2]: 6-cam x 1000-frame FTE (default_nolure: 20 keypoints, P = 26), shutter delay
  'const', interpolation 'vel' (the all_optimizations defaults,
  src/all_optimizations.py:127-136), initialised as core.fte does (src/core/fte.py:254-292):
  GPU pairwise triangulation of the nose, then the line fit.
* the FTE reprojection RMS of the parity metric (src/lib/metric.py:79-86: per observation
  |reprojection - measurement|, over the observations above the likelihood threshold; the
  3-D points are the per-camera shutter-shifted keypoints, src/lib/misc.py:126-141).
"""
from __future__ import annotations

import importlib
import os
from dataclasses import dataclass

import numpy as np

from . import _native, synth
from .kinematics import build_table

FTE_SEED = 77
FTE_TAU_MAX = 0.004


@dataclass
class FteWorkload:
    seq: object            # synth.Sequence (truth: x, pos3d, tau)
    scene: object          # synth.Scene
    cams: np.ndarray       # (C, 20) camera records
    meas: np.ndarray       # (N, C, L, 2), NaN -> 0
    w: np.ndarray          # (N, C, L): 1/R = 1/3 above the likelihood threshold, else 0
    X0: np.ndarray         # (N + 2, P) reference initialisation
    table: object          # kinematics table
    qinv: np.ndarray       # (P,) model weights
    nose_frames: np.ndarray
    nose_xyz: np.ndarray   # the triangulated nose the line fit used

    @property
    def Ts(self):
        return self.seq.Ts


def fte_workload(ctx, n_frames=1000, seed=FTE_SEED, mode='default_nolure', thresh=0.5) -> FteWorkload:
    """configs[2] (n_frames = 1000) / configs[3] (10,000) FTE input on the GPU context."""
    import pandas as pd
    cfte = importlib.import_module('acinoset_amd.core.fte')
    scene = synth.load_scene_file()
    seq = synth.make_sequence(n_frames, scene, mode=mode, seed=seed, tau_max=FTE_TAU_MAX)
    w = np.where(seq.likelihood > thresh, 1.0 / 3.0, 0.0)
    meas = np.nan_to_num(seq.uv)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    N = seq.uv.shape[0]
    valid = (seq.likelihood > thresh) & np.isfinite(seq.uv).all(-1)
    xyz, cnt = ctx.triangulate_dense(cams, seq.uv[:, :, 0], valid[:, :, 0])
    ok = cnt > 0
    nose_df = pd.DataFrame({'frame': np.arange(N)[ok], 'marker': 'nose', 'x': xyz[ok, 0], 'y': xyz[ok, 1],
                            'z': xyz[ok, 2]})
    X0 = cfte.initial_state(nose_df, mode, 0, N - 1)
    return FteWorkload(seq, scene, cams, meas, w, X0, build_table(mode), cfte.model_weights(mode),
                       np.arange(N)[ok], xyz[ok])


def fte_reproj_rms(ctx, wl: FteWorkload, X, tau, intermode=1):
    """Reprojection RMS (px) at an FTE solution over the observations with w > 0: the
    keypoints of every frame (GPU FK) shifted by the camera's shutter delay times the head
    velocity (intermode 'vel'; src/lib/misc.py:190-192), projected on the GPU."""
    X = np.asarray(X, np.float64)
    tau = np.asarray(tau, np.float64)
    N, C, L, _ = wl.meas.shape
    pos = ctx.fk(wl.table, np.ascontiguousarray(X[2:]))                       # (N, L, 3)
    vel = (X[2:, :3] - X[1:-1, :3]) / wl.Ts
    shift = vel[:, None, :] * (tau if tau.ndim == 2 else tau[None, :])[:, :, None]   # (N, C, 3)
    if intermode == 0:
        shift = np.zeros_like(shift)
    pts = pos[:, None] + shift[:, :, None]
    uv = np.stack([ctx.project(wl.cams, np.ascontiguousarray(pts[:, c].reshape(-1, 3)), np.full(N * L, c),
                               fte_form=True).reshape(N, L, 2) for c in range(C)], 1)
    m = wl.w > 0
    return float(np.sqrt(np.mean(np.sum((uv - wl.meas)[m] ** 2, -1))))


# ---- configs[1]: the reference's own 6-cam x 100-frame x 20-kp SBA run -------------------
REF_SBA_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden',
                               'sba_cfg2.npz')


@dataclass
class SbaWorkload:
    """The points-only SBA problem exactly as the reference built it (SURVEY config 2 =
    BASELINE configs[1]; `tests/golden/make_golden.py cfg2` ran the reference's
    `_sba_points`, src/lib/sba.py:285-313, on synth seed 0 and recorded its inputs, its
    triangulated initial points and its solution). Both layouts of the same problem:
    the reference's observation list and the dense slot-per-camera tensor."""
    K: np.ndarray
    D: np.ndarray
    R: np.ndarray
    t: np.ndarray
    cams: np.ndarray           # (C, 20)
    points_2d: np.ndarray      # (n_obs, 2) the reference's observation list
    point_idx: np.ndarray      # (n_obs,)
    cam_idx: np.ndarray        # (n_obs,)
    pts0: np.ndarray           # (n_pts, 3) the reference's triangulated start
    uv: np.ndarray             # (n_pts, C, 2) dense
    mask: np.ndarray           # (n_pts, C) u8
    ref_pts: np.ndarray        # (n_pts, 3) the reference's solution
    ref_resid_after: np.ndarray  # (2 n_obs,) the reference's residuals at its solution
    truth: np.ndarray          # (n_pts, 3) synthetic truth of every point
    n_frames: int

    @property
    def n_points(self):
        return len(self.pts0)


def sba_reference_workload() -> SbaWorkload:
    d = np.load(REF_SBA_FIXTURE, allow_pickle=False)
    K, D, R, t = d['K'], d['D'], d['R'], d['t']
    C = len(K)
    # C order throughout: the fixture's arrays came out of DataFrames (column-major) and the
    # bench hands their device copies to the C ABI as raw pointers
    c64 = lambda a: np.ascontiguousarray(a, np.float64)  # noqa: E731
    p2 = c64(d['points_2d'])
    pi = np.ascontiguousarray(d['point_indices'], np.int64)
    ci = np.ascontiguousarray(d['camera_indices'], np.int64)
    pts0 = c64(d['points_3d'])
    n = len(pts0)
    uv = np.zeros((n, C, 2))
    mask = np.zeros((n, C), np.uint8)
    if np.any(np.bincount(pi * C + ci, minlength=n * C) > 1):
        raise ValueError('a point has two observations from one camera: no dense layout')
    uv[pi, ci] = p2
    mask[pi, ci] = 1
    n_frames = int(d['n_frames'])
    scene = synth.Scene(K, D, R, t, tuple(int(v) for v in d['res']))
    seq = synth.make_sequence(n_frames, scene, mode='default_nolure', seed=0)
    truth = seq.pos3d[:, 0][d['pts_frame'], d['pts_marker']]
    return SbaWorkload(c64(K), c64(D), c64(R), c64(t), _native.pack_cameras(K, D, R, t), p2, pi, ci, pts0, uv, mask,
                       c64(d['pts_out']), c64(d['resid_after']), c64(truth), n_frames)


def reproj_rms(resid):
    """RMS over observations of |reprojection - observation| (px), from the interleaved
    (u, v) residual vector of `cost_func_points_only` (src/lib/sba.py:149-153)."""
    r = np.asarray(resid, np.float64).reshape(-1, 2)
    return float(np.sqrt(np.mean(np.sum(r * r, 1))))
