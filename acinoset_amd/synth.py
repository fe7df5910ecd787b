"""Synthetic AcinoSet-like sequences.

There is no dataset on the GPU box, so every benchmark and most tests run on
seeded synthetic sequences:

* scene: `configs/dummy_scene.json` of the reference (6 fisheye cameras in a ring,
  2704x1520), copied as data to `acinoset_amd/data/dummy_scene.json`; a 12-camera
  ring with the same K/D is synthesised for config 5;
* subject: the cheetah tree of `acinoset_amd.kinematics` (20 keypoints =
  `default_nolure`, P = 26; `head` for the reference's default FTE run);
  the root runs along +x through the scene centre, joint angles are smooth gait
  sinusoids plus a small random walk;
* observations: fisheye projection + N(0, 1 px) noise, likelihood 0.99, 5 %
  dropout (likelihood 0.1), 1 % outliers of +-30 px, points outside the image
  dropped (likelihood 0).

This module only *makes inputs* (ground truth via a host FK and projection);
no solve ever runs through it.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .kinematics import fk_numpy, get_markers, get_pose_params

DATA_DIR = os.path.join(os.path.dirname(__file__), 'data')
DUMMY_SCENE = os.path.join(DATA_DIR, 'dummy_scene.json')


@dataclass
class Scene:
    K: np.ndarray      # (C,3,3)
    D: np.ndarray      # (C,4,1)
    R: np.ndarray      # (C,3,3)
    t: np.ndarray      # (C,3,1)
    res: tuple

    @property
    def n_cams(self) -> int:
        return len(self.K)

    def camera_params(self):
        """The reference's `camera_params` tuple (`src/all_optimizations.py:68`)."""
        return (self.K, self.D, self.R, self.t, self.res, self.n_cams)

    def subset(self, cams):
        cams = list(cams)
        return Scene(self.K[cams], self.D[cams], self.R[cams], self.t[cams], self.res)

    def to_json(self, path):
        cams = [{'k': k.tolist(), 'd': d.tolist(), 'r': r.tolist(), 't': t.tolist()}
                for k, d, r, t in zip(self.K, self.D, self.R, self.t)]
        with open(path, 'w') as f:
            json.dump({'camera_resolution': list(self.res), 'cameras': cams}, f)


def load_scene_file(path: str = DUMMY_SCENE) -> Scene:
    with open(path) as f:
        d = json.load(f)
    K = np.array([c['k'] for c in d['cameras']], np.float64)
    D = np.array([c['d'] for c in d['cameras']], np.float64).reshape(-1, 4, 1)
    R = np.array([c['r'] for c in d['cameras']], np.float64)
    t = np.array([c['t'] for c in d['cameras']], np.float64).reshape(-1, 3, 1)
    return Scene(K, D, R, t, tuple(d['camera_resolution']))


def ring_scene(n_cams: int = 12, radius: float = 6.5, centre=(1.9, 6.4), seed: int = 4) -> Scene:
    """Ring of `n_cams` cameras with the dummy scene's K/D looking at `centre`."""
    base = load_scene_file()
    rng = np.random.default_rng(seed)
    K = np.repeat(base.K[:1], n_cams, 0)
    D = np.repeat(base.D[:1], n_cams, 0)
    Rs, ts = [], []
    for i in range(n_cams):
        ang = 2 * np.pi * i / n_cams
        c = np.array([centre[0] + radius * np.cos(ang), centre[1] + radius * np.sin(ang),
                      rng.uniform(0.3, 0.5)])
        target = np.array([centre[0], centre[1], 0.5])
        z = target - c
        z /= np.linalg.norm(z)
        x = np.cross(z, [0.0, 0.0, 1.0])
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R = np.stack([x, y, z])
        Rs.append(R)
        ts.append((-R @ c).reshape(3, 1))
    return Scene(K, D, np.array(Rs), np.array(ts), base.res)


def project_numpy(pts: np.ndarray, K, D, R, t) -> np.ndarray:
    """Fisheye projection (the model of `src/core/fte.py:80-96`) for data generation."""
    Xc = pts @ R.T + t.reshape(1, 3)
    a = Xc[:, 0] / Xc[:, 2]
    b = Xc[:, 1] / Xc[:, 2]
    r = np.sqrt(a * a + b * b)
    th = np.arctan(r)
    d = D.ravel()
    th2 = th * th
    thd = th * (1 + th2 * (d[0] + th2 * (d[1] + th2 * (d[2] + th2 * d[3]))))
    s = np.where(r > 1e-8, thd / np.where(r > 1e-8, r, 1.0), 1.0)
    u = K[0, 0] * a * s + K[0, 2]
    v = K[1, 1] * b * s + K[1, 2]
    out = np.stack([u, v], -1)
    out[Xc[:, 2] <= 0] = np.nan
    return out


@dataclass
class Sequence:
    scene: Scene
    mode: str
    markers: list
    Ts: float
    x: np.ndarray           # (N, P) ground-truth pose parameters
    tau: np.ndarray         # (C,) ground-truth shutter delays (tau[0] = 0)
    pos3d: np.ndarray       # (N, C, L, 3) ground-truth marker positions seen by each camera
    uv: np.ndarray          # (N, C, L, 2) observations (NaN where not visible)
    likelihood: np.ndarray  # (N, C, L)

    @property
    def N(self):
        return self.x.shape[0]

    def to_df(self, start_frame: int = 0):
        """Long DataFrame [frame, camera, marker, x, y, likelihood] as produced by
        `load_dlc_points_as_df` (`src/lib/utils.py:142-148`)."""
        import pandas as pd
        N, C, L, _ = self.uv.shape
        f, c, l = np.meshgrid(np.arange(N) + start_frame, np.arange(C), np.arange(L), indexing='ij')
        df = pd.DataFrame({
            'frame': f.ravel().astype(np.int64),
            'camera': c.ravel().astype(np.int64),
            'marker': np.array(self.markers, dtype=object)[l.ravel()],
            'x': self.uv[..., 0].ravel(),
            'y': self.uv[..., 1].ravel(),
            'likelihood': self.likelihood.ravel(),
        })
        return df.sort_values(['camera', 'frame'], kind='stable').reset_index(drop=True)


def make_sequence(n_frames: int, scene: Optional[Scene] = None, mode: str = 'default_nolure',
                  fps: float = 90.0, noise_px: float = 1.0, dropout: float = 0.05,
                  outliers: float = 0.01, tau_max: float = 0.0, speed: Optional[float] = None,
                  gait_amp: float = 0.2, seed: int = 0, drift: float = 1.0) -> Sequence:
    """Seeded synthetic sequence per SURVEY.md §8(d). `gait_amp` (rad) and `drift` (a factor on
    the joint angles' random-walk drift) set how far the joints move from zero."""
    scene = scene or load_scene_file()
    idx = get_pose_params(mode)
    markers = get_markers(mode)
    P, L, C, N = len(idx), len(markers), scene.n_cams, n_frames
    Ts = 1.0 / fps
    drift_scale = drift
    rng0 = np.random.default_rng(seed)
    t = np.arange(N) * Ts
    if speed is None:
        speed = min(4.5, 4.0 / max(N * Ts, 1e-9))
    x = np.zeros((N, P))
    x[:, idx['x_0']] = 1.9 + speed * (t - 0.5 * N * Ts)
    x[:, idx['y_0']] = 6.4 + 0.05 * np.sin(2 * np.pi * 0.5 * t)
    x[:, idx['z_0']] = 0.6 + 0.03 * np.sin(2 * np.pi * 2.0 * t)
    gait = 2 * np.pi * 2.0 * t
    for name, i in idx.items():
        if name in ('x_0', 'y_0', 'z_0'):
            continue
        if name == 'l_1':
            x[:, i] = 0.28
            continue
        if name in ('x_l', 'y_l', 'z_l'):
            base = {'x_l': 1.9, 'y_l': 6.4, 'z_l': 0.1}[name]
            x[:, i] = base + (x[:, idx['x_0']] - 1.9 + 2.0 if name == 'x_l' else 0.0)
            continue
        amp = gait_amp if name.startswith('theta_') and int(name.split('_')[1]) >= 6 else 0.25 * gait_amp
        phase = rng0.uniform(0, 2 * np.pi)
        walk = np.cumsum(rng0.normal(0, 0.05 * np.sqrt(Ts), N))
        x[:, i] = amp * np.sin(gait + phase) + 0.2 * drift_scale * walk
    tau = np.zeros(C)
    if tau_max > 0:
        tau[1:] = rng0.uniform(-tau_max, tau_max, C - 1)
    # velocity of the head for the shutter shift (backward difference, as FTE's dx)
    dx = np.zeros((N, 3))
    dx[1:] = (x[1:, :3] - x[:-1, :3]) / Ts
    dx[0] = dx[1] if N > 1 else 0.0
    pos3d = np.zeros((N, C, L, 3))
    uv = np.zeros((N, C, L, 2))
    for c in range(C):
        pos = fk_numpy(mode, x)
        pos = pos + (dx * tau[c])[:, None, :]
        pos3d[:, c] = pos
        uv[:, c] = project_numpy(pos.reshape(-1, 3), scene.K[c], scene.D[c], scene.R[c],
                                 scene.t[c]).reshape(N, L, 2)
    rng1 = np.random.default_rng(seed + 1)
    uv = uv + rng1.normal(0.0, noise_px, uv.shape)
    lik = np.full((N, C, L), 0.99)
    rng2 = np.random.default_rng(seed + 2)
    lik[rng2.random((N, C, L)) < dropout] = 0.1
    rng3 = np.random.default_rng(seed + 3)
    om = rng3.random((N, C, L)) < outliers
    uv[om] += rng3.choice([-30.0, 30.0], size=(int(om.sum()), 2))
    W, H = scene.res
    vis = np.isfinite(uv).all(-1) & (uv[..., 0] >= 0) & (uv[..., 0] < W) & (uv[..., 1] >= 0) & (uv[..., 1] < H)
    uv[~vis] = np.nan
    lik[~vis] = 0.0
    return Sequence(scene, mode, markers, Ts, x, tau, pos3d, uv, lik)


def dense_sba_problem(seq: Sequence, thresh: float = 0.5, init_noise_m: float = 0.02, seed: int = 7):
    """Dense SBA problem on the (frame, marker) grid: one point per (frame, marker)
    seen by >= 2 cameras. Returns (uv (n_pts, C, 2), mask (n_pts, C) u8,
    pts0 (n_pts, 3), pt_truth (n_pts, 3), keep (N*L,) bool).

    `pts0` is the truth perturbed by N(0, init_noise_m) — a stand-in for the
    pairwise-triangulation init of `src/lib/sba.py:290`.
    """
    N, C, L, _ = seq.uv.shape
    valid = (seq.likelihood > thresh) & np.isfinite(seq.uv).all(-1)      # (N,C,L)
    v = valid.transpose(0, 2, 1).reshape(N * L, C)                         # (N*L, C)
    keep = v.sum(1) >= 2
    uv = seq.uv.transpose(0, 2, 1, 3).reshape(N * L, C, 2)[keep]
    mask = v[keep].astype(np.uint8)
    uv = np.where(mask[..., None] > 0, uv, 0.0)
    truth = seq.pos3d[:, 0].reshape(N * L, 3)[keep]
    rng = np.random.default_rng(seed)
    pts0 = truth + rng.normal(0.0, init_noise_m, truth.shape)
    return np.ascontiguousarray(uv), np.ascontiguousarray(mask), pts0, truth, keep
