"""GPU: the FTE's assembled block-tridiagonal normal matrix.

acs_fte_debug_blocks returns the damped 3-frame super-blocks D_i as k_cr_assemble_build forms
them (levels = 0) or as the cyclic reduction leaves them for the next level (levels = L).

* The assembled D equals the dense normal matrix of acs_fte_eval (the linearisation the
  parity tests pin to the reference model) bit for bit, and is bitwise symmetric at the
  configs[2] and configs[3] sizes: element (r, c) and (c, r) are one banded-row entry.
* So the single-GPU solve stores D as its upper 16 x 16 tiles and levels 0-1 read the lower
  ones transposed (k_cr_level DUP): that solve, and the blocks after 2 levels, equal the
  whole-D form (ACS_D_FULL=1, read once per process: a child process) bit for bit.
  (Round 5's attempt at this moved the 10,000-frame cost by 2e-8: the survivor apply read the
  lower half from the upper tiles that other waves of its workgroup were overwriting; it now
  holds a barrier between its reads and its stores.)
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import fte as ofte
from acinoset_amd import _native, kinematics as pkin, synth, workloads

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _small(N=40):
    scene = synth.load_scene_file()
    seq = synth.make_sequence(N, scene, mode='default_nolure', seed=2, tau_max=0.004)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem('default_nolure', seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=True,
                        intermode='vel')
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    return prob, cams, X0


def test_fte_assembled_blocks_equal_dense_normal_matrix(ctx):
    prob, cams, X0 = _small()
    table = pkin.build_table('default_nolure')
    P = table.P
    tau = np.zeros(len(cams))
    D, _ = ctx.fte_debug_blocks(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, tau, lam=0.0, levels=0)
    _, _, H = ctx.fte_eval(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, tau)
    M = X0.shape[0]
    nblk, BP = D.shape[:2]
    for i in range(nblk):
        f0, f1 = 3 * i, min(3 * i + 3, M)
        n = (f1 - f0) * P
        np.testing.assert_array_equal(D[i, :n, :n], H[f0 * P:f0 * P + n, f0 * P:f0 * P + n])
        assert np.array_equal(D[i, n:, n:], np.eye(BP - n))       # padding rows: identity


@pytest.mark.parametrize('N', [1000, 10000])
def test_fte_assembled_blocks_bitwise_symmetric(ctx, N):
    wl = workloads.fte_workload(ctx, N)
    D, _ = ctx.fte_debug_blocks(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0, np.zeros(len(wl.cams)),
                                lam=1e-3, levels=0)
    assert np.isfinite(D).all()
    bad = np.nonzero((D != np.swapaxes(D, 1, 2)).any((1, 2)))[0]
    assert len(bad) == 0, f'{len(bad)} of {len(D)} assembled blocks not bitwise symmetric, first {bad[:5]}'


def test_fte_upper_tile_d_equals_whole_d(ctx, tmp_path):
    N = 1000
    wl = workloads.fte_workload(ctx, N)
    tau = np.zeros(len(wl.cams))
    X, t, rep = ctx.fte_solve(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0)
    D2, L = ctx.fte_debug_blocks(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0, tau, lam=1e-3, levels=2)
    assert L == 2
    code = f"""
import sys, numpy as np
sys.path.insert(0, {os.path.dirname(HERE)!r})
from acinoset_amd import _native, workloads
ctx = _native.Context(0)
wl = workloads.fte_workload(ctx, {N})
X, t, rep = ctx.fte_solve(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0)
D2, L = ctx.fte_debug_blocks(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0, np.zeros(len(wl.cams)),
                             lam=1e-3, levels=2)
np.savez({str(tmp_path / 'full.npz')!r}, X=X, t=t, iters=rep['iters'], D2=D2[::4])
"""
    env = dict(os.environ, ACS_D_FULL='1')
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    full = np.load(tmp_path / 'full.npz')
    assert int(full['iters']) == rep['iters']
    np.testing.assert_array_equal(X, full['X'])
    np.testing.assert_array_equal(t, full['t'])
    np.testing.assert_array_equal(D2[::4], full['D2'])
