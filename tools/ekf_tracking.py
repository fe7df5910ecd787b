"""EKF tracking study on the bench's synthetic sequences: does the filter (the reference's
model, src/core/ekf.py) track the truth, per camera count / skeleton / numerics mode?
Prints one line per case: keypoint RMS of x_est / x_smooth vs the truth, outlier fraction.
Run on a GPU box: python tools/ekf_tracking.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acinoset_amd import _native, synth  # noqa: E402
import importlib  # noqa: E402
cekf = importlib.import_module('acinoset_amd.core.ekf')
from acinoset_amd.kinematics import build_table  # noqa: E402
from oracle.kinematics import marker_positions  # noqa: E402


def case(ctx, n_cams, mode, n_frames, ref_numerics, n_seq=4, p0_abs=False):
    scene = synth.load_scene_file() if n_cams == 6 else synth.ring_scene(n_cams)
    seqs = [synth.make_sequence(n_frames, scene, mode=mode, seed=500 + k) for k in range(n_seq)]
    table = build_table(mode)
    P = table.P
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    meas = np.stack([q.uv for q in seqs])
    lik = np.stack([q.likelihood for q in seqs])
    s0 = np.zeros((n_seq, 3 * P))
    for k, q in enumerate(seqs):
        s0[k, :P] = q.x[0]
        s0[k, P:2 * P] = (q.x[1] - q.x[0]) / q.Ts
    P0 = cekf.initial_covariance(mode)
    if p0_abs:  # the reference's P0 carries a negative variance (neck length, src/core/ekf.py)
        P0 = np.abs(P0)
    covs = (cekf.CAL_COVS * ((n_cams + 5) // 6))[:n_cams]
    out = ctx.ekf_run(table, cams, meas, lik, 90.0, 0.5, float(scene.res[0]), cekf.measurement_std(n_cams, covs),
                      cekf.process_covariance(P, 1 / 90.0), P0, s0,
                      ref_numerics=ref_numerics)
    res = []
    for key in ('x_est', 'x_smooth'):
        e = []
        for k, q in enumerate(seqs):
            pe = marker_positions(mode, out[key][k][:, :P])
            pt = marker_positions(mode, q.x)
            e.append(np.sqrt(np.mean(np.sum((pe - pt) ** 2, -1), -1)))
        e = np.array(e)                                    # (S, N)
        res.append((float(np.median(e[:, :50])), float(np.median(e[:, -50:])), float(e.max())))
    nobs = np.sum(lik > 0.5) * 2 / n_seq
    print(f'C={n_cams:2d} {mode:8s} N={n_frames:4d} ref={int(ref_numerics)} p0abs={int(p0_abs)}  est rms first50 {res[0][0]:.4f} '
          f'last50 {res[0][1]:.4f} max {res[0][2]:.3g} | smooth first50 {res[1][0]:.4f} last50 {res[1][1]:.4f} '
          f'| outliers/seq {np.mean(out["outliers"]):.0f} of {nobs:.0f}', flush=True)


if __name__ == '__main__':
    ctx = _native.Context(0)
    for n_cams in (6, 12):
        for p0_abs in (False, True):
            case(ctx, n_cams, 'default', 500, True, p0_abs=p0_abs)
    case(ctx, 12, 'default', 500, False, p0_abs=True)
    case(ctx, 6, 'head', 500, True)
