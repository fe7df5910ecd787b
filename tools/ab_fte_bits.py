"""Bit-for-bit A/B of FTE solves between two builds of the library (ACINOSET_HIP_LIB picks the
one under test): python tools/ab_fte_bits.py save TAG  (writes gpurun_out/fte_bits_TAG.npz),
python tools/ab_fte_bits.py cmp TAG_A TAG_B. Cases: the single-GPU solve at 1,000 and 10,000
frames (const delays), the variable-delay solve at 300 frames, the 3-window virtual
frame-window solve at 600 frames and the 2-window one at 4,000 frames."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gpurun_out')


def save(tag):
    import bench
    from acinoset_amd import _native, dist
    ctx = _native.Context(0)
    res = {}
    for n in (1000, 10000):
        seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, n)
        X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0)
        res[f'X{n}'], res[f'tau{n}'], res[f'it{n}'] = X, tau, np.array([rep['iters']])
    seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, 300)
    X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0, sd_mode='variable')
    res['Xvar'], res['tauvar'] = X, tau
    seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, 600)
    X, tau, rep = dist.fte_solve_virtual(ctx, table, cams, meas, w, seq.Ts, qinv, X0, world=3)
    res['Xwin'], res['tauwin'] = X, tau
    # 2 windows of 4,000 frames: 667 super-blocks per rank, more than two rounds of the CUs
    # (the 512-thread compact-row assembly with the ranks' raw diagonals)
    seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, 4000)
    X, tau, rep = dist.fte_solve_virtual(ctx, table, cams, meas, w, seq.Ts, qinv, X0, world=2)
    res['Xwin2'], res['tauwin2'] = X, tau
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f'fte_bits_{tag}.npz'), **res)
    print(tag, {k: (v.shape, float(np.abs(v).sum())) for k, v in res.items()})


def cmp(a, b):
    A = np.load(os.path.join(OUT, f'fte_bits_{a}.npz'))
    B = np.load(os.path.join(OUT, f'fte_bits_{b}.npz'))
    ok = True
    for k in A.files:
        same = np.array_equal(A[k], B[k])
        ok &= same
        print(f'{k:8s} bitwise {"equal" if same else "DIFFERENT"}  max|d| {float(np.abs(A[k] - B[k]).max()):.3e}')
    print('ALL BITWISE EQUAL' if ok else 'DIFFERENCES')
    return ok


if __name__ == '__main__':
    if sys.argv[1] == 'save':
        save(sys.argv[2])
    else:
        sys.exit(0 if cmp(sys.argv[2], sys.argv[3]) else 1)
