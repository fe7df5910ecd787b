"""GPU parity of the multi-GPU solves: frame-window FTE (acs_fte_dist_*)
and points + extrinsics SBA (acs_sba_ext_dist_*, same tolerances as the single-GPU
extrinsics parity: cost 1e-12 relative, points 1e-9 m, rotations 1e-10).

* `fte_solve_virtual`: W ranks emulated in one process on one GPU (payload sums in rank
  order) must reproduce the single-GPU acs_fte_solve iterate for iterate: same iteration
  count and status, X within 1e-9, tau within 1e-12 s, cost 1e-11 relative (the
  decomposition only reorders sums).
* one LM step of the distributed HIP path against the oracle restatement of the same
  decomposition (oracle/fte_dist.py): 1e-9.
* world_size 2 through torch.distributed (gloo on the device tensors; the multi-GPU run
  uses the same calls over RCCL): two processes on the one GPU reach the same result.
"""
import os
import socket

import numpy as np
import pytest

from oracle import fte as ofte, fte_dist as odist
from acinoset_amd import _native, dist, kinematics as pkin, synth

pytestmark = pytest.mark.gpu


def _problem(N, mode='default_nolure', sd=True, inter='vel', seed=2, sd_mode='const', n_cams=None):
    scene = synth.load_scene_file() if n_cams is None else synth.ring_scene(n_cams)
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed, tau_max=0.004 if sd else 0.0)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem(mode, seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=sd, intermode=inter,
                        sd_mode=sd_mode)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    return prob, cams, X0


@pytest.mark.parametrize('mode,N,sd,inter', [('default_nolure', 40, True, 'vel'), ('head', 61, True, 'acc'),
                                             ('default_nolure', 31, False, 'pos')])
@pytest.mark.parametrize('world', [2, 3, 8])
def test_fte_dist_virtual_matches_single(ctx, mode, N, sd, inter, world):
    prob, cams, X0 = _problem(N, mode, sd, inter)
    table = pkin.build_table(mode)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, shutter_delay=sd,
                               intermode=prob.im)
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                        shutter_delay=sd, intermode=prob.im, world=world)
    assert rd['iters'] == r1['iters'] and rd['n_accepted'] == r1['n_accepted'], (rd, r1)
    assert rd['status'] == r1['status'] and rd['n_bad_pivots'] == 0
    assert abs(rd['cost_after'] - r1['cost_after']) <= 1e-11 * r1['cost_after']
    np.testing.assert_allclose(Xd, X1, rtol=0, atol=1e-9)
    np.testing.assert_allclose(td, t1, rtol=0, atol=1e-12)


@pytest.mark.parametrize('n_cams,mode', [(12, 'default_nolure'), (16, 'default_nolure'), (16, 'default')])
def test_fte_dist_virtual_many_cameras_matches_single(ctx, n_cams, mode):
    """Frame windows with a ring of 12 / 16 cameras (synth.ring_scene): a tau border of 16
    constant delays takes two GB column-blocks (GR = 32) in every rank's reduction and in the
    reduced system; 'default' the 96-row super-blocks. 3 ranks against the single-GPU solve."""
    prob, cams, X0 = _problem(30, mode, n_cams=n_cams)
    table = pkin.build_table(mode)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, intermode=prob.im)
    assert r1['status_name'] in ('ftol', 'xtol', 'gtol'), r1
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                        intermode=prob.im, world=3)
    assert rd['iters'] == r1['iters'] and rd['n_accepted'] == r1['n_accepted'], (rd, r1)
    assert rd['status'] == r1['status'] and rd['n_bad_pivots'] == 0
    assert abs(rd['cost_after'] - r1['cost_after']) <= 1e-11 * r1['cost_after']
    np.testing.assert_allclose(Xd, X1, rtol=0, atol=1e-9)
    np.testing.assert_allclose(td, t1, rtol=0, atol=1e-12)


@pytest.mark.parametrize('mode,N,inter', [('default_nolure', 40, 'vel'), ('head', 47, 'acc')])
@pytest.mark.parametrize('world', [2, 3, 8])
def test_fte_dist_virtual_variable_delays_matches_single(ctx, mode, N, inter, world):
    """shutter_delay_mode='variable' over frame windows: each frame's delays eliminated and
    stepped by the rank owning the frame, gathered once with the rows. Same iterates as the
    single-GPU solve (which eliminates them in one pass)."""
    prob, cams, X0 = _problem(N, mode, True, inter, sd_mode='variable')
    table = pkin.build_table(mode)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, intermode=prob.im,
                               sd_mode='variable')
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                        intermode=prob.im, world=world, sd_mode='variable')
    assert td.shape == (N, 6)
    assert rd['iters'] == r1['iters'] and rd['n_accepted'] == r1['n_accepted'], (rd, r1)
    assert rd['status'] == r1['status'] and rd['n_bad_pivots'] == 0
    assert abs(rd['cost_after'] - r1['cost_after']) <= 1e-11 * r1['cost_after']
    np.testing.assert_allclose(Xd, X1, rtol=0, atol=1e-9)
    np.testing.assert_allclose(td, t1, rtol=0, atol=1e-12)


def test_fte_dist_variable_delays_matches_oracle_decomposition(ctx):
    """The variable-delay rank protocol on the GPU against its numpy restatement
    (oracle/fte_dist.py), 3 ranks, full solve: 1e-9."""
    prob, cams, X0 = _problem(30, 'head', True, 'vel', sd_mode='variable')
    table = pkin.build_table('head')
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, world=3,
                                        sd_mode='variable')
    ranks = [odist.OracleFteRank(prob, X0, None, r, 3) for r in range(3)]
    dist.lm_loop(ranks, dist.local_allreduce)
    Xo, to, io = ranks[0].result()
    assert rd['iters'] == io['iters']
    np.testing.assert_allclose(Xd, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(td, to, rtol=0, atol=1e-11)


@pytest.mark.parametrize('world', [2, 5])
def test_fte_dist_one_step_matches_oracle_decomposition(ctx, world):
    prob, cams, X0 = _problem(40)
    table = pkin.build_table(prob.mode)
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                        opts=ctx.fte_default_opts(max_iters=1), world=world)
    ranks = [odist.OracleFteRank(prob, X0, None, r, world, max_iters=1) for r in range(world)]
    dist.lm_loop(ranks, dist.local_allreduce)
    Xo, to, io = ranks[0].result()
    assert rd['n_accepted'] == io['n_accepted'] == 1
    np.testing.assert_allclose(Xd, Xo, rtol=0, atol=1e-9)
    np.testing.assert_allclose(td, to, rtol=0, atol=1e-12)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ctx = _native.Context(0)
        prob, cams, X0 = _problem(40)
        table = pkin.build_table(prob.mode)
        X, tau, rep = dist.fte_solve_dist(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
        np.savez(os.path.join(out_dir, f'rank{rank}.npz'), X=X, tau=tau, iters=rep['iters'])
        del torch
    finally:
        tdist.destroy_process_group()


def test_fte_dist_two_processes(ctx, tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method='spawn')
    prob, cams, X0 = _problem(40)
    table = pkin.build_table(prob.mode)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    a, b = (np.load(tmp_path / f'rank{r}.npz') for r in range(2))
    assert np.array_equal(a['X'], b['X']) and np.array_equal(a['tau'], b['tau'])
    assert int(a['iters']) == r1['iters']
    np.testing.assert_allclose(a['X'], X1, rtol=0, atol=1e-9)


# ---- points + extrinsics SBA over ranks ------------------------------------------------
def _ext():
    from conftest import golden
    g = golden('sba_extrinsics')
    return g, _native.pack_cameras(g['K'], g['D'], g['R0'], g['t0'])


@pytest.mark.parametrize('world', [2, 3, 8])
def test_sba_ext_dist_virtual_matches_single(ctx, world):
    g, cams = _ext()
    o = ctx.sba_ext_opts(max_iters=200)
    c1, X1, _, _, r1 = ctx.sba_extrinsics(cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                          g['points_3d'], o)
    cd, Xd, rd = dist.sba_extrinsics_virtual(ctx, cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                             g['points_3d'], o, world=world)
    assert rd['iters'] == r1['iters'] and rd['n_accepted'] == r1['n_accepted'] and rd['status'] == r1['status']
    assert abs(rd['cost_after'] - r1['cost_after']) <= 1e-12 * r1['cost_after']
    np.testing.assert_allclose(Xd, X1, rtol=0, atol=1e-9)
    np.testing.assert_allclose(cd[:, 8:17], c1[:, 8:17], rtol=0, atol=1e-10)
    np.testing.assert_allclose(cd[:, 17:], c1[:, 17:], rtol=0, atol=1e-9)


def test_dist_max_iters_zero_takes_no_step(ctx):
    """max_iters = 0 over ranks: no step (X0 back, iters 0), as acs_fte_solve /
    acs_sba_extrinsics - the first round stops before stepping."""
    prob, cams, X0 = _problem(31, 'head', True, 'vel')
    table = pkin.build_table('head')
    o = ctx.fte_default_opts(max_iters=0)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, shutter_delay=True,
                               intermode=prob.im, opts=o)
    Xd, td, rd = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                        shutter_delay=True, intermode=prob.im, opts=o, world=2)
    assert r1['iters'] == 0 and rd['iters'] == 0, (r1, rd)
    np.testing.assert_array_equal(Xd, X1)
    g, cams = _ext()
    oe = ctx.sba_ext_opts(max_iters=0)
    cd, Xe, re_ = dist.sba_extrinsics_virtual(ctx, cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                              g['points_3d'], oe, world=2)
    assert re_['iters'] == 0
    np.testing.assert_array_equal(Xe, g['points_3d'])


def _ext_worker(rank, world, port, out_dir):
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ctx = _native.Context(0)
        g, cams = _ext()
        c, X, rep = dist.sba_extrinsics_dist(ctx, cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                             g['points_3d'], ctx.sba_ext_opts(max_iters=200))
        np.savez(os.path.join(out_dir, f'ext{rank}.npz'), cams=c, X=X, iters=rep['iters'])
    finally:
        tdist.destroy_process_group()


def test_sba_ext_dist_two_processes(ctx, tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_ext_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method='spawn')
    g, cams = _ext()
    c1, X1, _, _, r1 = ctx.sba_extrinsics(cams, g['points_2d'], g['point_indices'], g['camera_indices'],
                                          g['points_3d'], ctx.sba_ext_opts(max_iters=200))
    a, b = (np.load(tmp_path / f'ext{r}.npz') for r in range(2))
    assert np.array_equal(a['cams'], b['cams']) and np.array_equal(a['X'], b['X'])
    assert int(a['iters']) == r1['iters']
    np.testing.assert_allclose(a['X'], X1, rtol=0, atol=1e-9)


def test_fte_dist_device_resident_inputs_match_host_inputs(ctx):
    """HipFteRank with the inputs already in HBM (ACS_DEVICE_PTRS, copied device to device
    into each rank) gives the solve of the host-input ranks, bit for bit."""
    import torch
    prob, cams, X0 = _problem(40)
    table = pkin.build_table(prob.mode)
    dv = torch.device('cuda', ctx.device)
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dv, dt)  # noqa: E731
    dev = dict(ints=T(table.ints, torch.int32), reals=T(table.reals), cams=T(cams), meas=T(np.nan_to_num(prob.meas)),
               w=T(prob.w), qinv=T(prob.qinv), X=T(X0), tau=torch.zeros(len(cams), dtype=torch.float64, device=dv))
    outs = []
    with dist._on_torch_stream(ctx):
        for use_dev in (False, True):
            ranks = [dist.HipFteRank(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, rank=r, world=2,
                                     dev=dev if use_dev else None) for r in range(2)]
            try:
                dist.lm_loop(ranks, dist.local_allreduce)
                outs.append(ranks[0].result())
            finally:
                for r in ranks:
                    r.close()
    (Xh, th, rh), (Xd, td, rd) = outs
    assert rh['iters'] == rd['iters'] and rh['n_accepted'] == rd['n_accepted']
    np.testing.assert_array_equal(Xd, Xh)
    np.testing.assert_array_equal(td, th)


def test_fte_dist_reset_reuses_handles_without_allocation(ctx):
    """acs_fte_dist_reset: a second solve on the same rank handles (3 virtual ranks), restarted
    from device tensors, repeats the first one bit for bit and makes no device or pinned-host
    allocation (acs_alloc_events unchanged: the bench's timed multi-GPU solves reuse one handle
    per rank); a reset to another start equals fresh handles created from that start."""
    import torch
    prob, cams, X0 = _problem(40)
    table = pkin.build_table(prob.mode)
    dv = torch.device('cuda', ctx.device)
    X1 = X0 + 1e-3 * np.random.default_rng(5).standard_normal(X0.shape)
    with dist._on_torch_stream(ctx):
        ranks = [dist.HipFteRank(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0, rank=r, world=3)
                 for r in range(3)]
        try:
            dist.lm_loop(ranks, dist.local_allreduce)
            Xa, ta, ra = ranks[0].result()
            dX = torch.from_numpy(np.ascontiguousarray(X0)).to(dv)
            dt = torch.zeros(len(cams), dtype=torch.float64, device=dv)
            oX = torch.empty_like(dX)
            otau = torch.empty_like(dt)
            a0 = _native.alloc_events()
            for r in ranks:
                r.reset(dX, dt)
            dist.lm_loop(ranks, dist.local_allreduce)
            _, _, rb = ranks[0].result(oX, otau)
            torch.cuda.synchronize()
            assert _native.alloc_events() == a0
            assert rb['iters'] == ra['iters'] and rb['n_accepted'] == ra['n_accepted']
            np.testing.assert_array_equal(oX.cpu().numpy(), Xa)
            np.testing.assert_array_equal(otau.cpu().numpy(), ta)
            for r in ranks:                                   # host-array reset to another start
                r.reset(X1)
            dist.lm_loop(ranks, dist.local_allreduce)
            Xc, tc, rc = ranks[0].result()
        finally:
            for r in ranks:
                r.close()
    Xf, tf, rf = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X1, world=3)
    assert rc['iters'] == rf['iters'] and rc['n_accepted'] == rf['n_accepted']
    np.testing.assert_array_equal(Xc, Xf)
    np.testing.assert_array_equal(tc, tf)


def test_fte_dist_chain_back_launch_equals_per_level_launches(ctx, tmp_path):
    """k_cr_back_chain (a rank chain's back substitution and trial rows in one launch) against
    the round-5 form (one k_cr_back launch per level + k_cr_trial, forced by
    ACS_DIST_BACK_LEVELS=1, read once per process: a child process): 3 and 8 virtual ranks,
    the same iterations and bit-identical X and tau (same sums in the same order)."""
    import subprocess
    import sys
    prob, cams, X0 = _problem(61, 'head', True, 'acc')
    table = pkin.build_table('head')
    ours = {}
    for world in (3, 8):
        ours[world] = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                             intermode=prob.im, world=world)
    here = os.path.dirname(os.path.abspath(__file__))
    code = f"""
import sys, numpy as np
sys.path.insert(0, {os.path.dirname(here)!r}); sys.path.insert(0, {here!r})
from test_gpu_dist import _problem
from acinoset_amd import _native, dist, kinematics as pkin
ctx = _native.Context(0)
prob, cams, X0 = _problem(61, 'head', True, 'acc')
table = pkin.build_table('head')
out = {{}}
for world in (3, 8):
    X, tau, rep = dist.fte_solve_virtual(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                         intermode=prob.im, world=world)
    out[f'X{{world}}'] = X; out[f't{{world}}'] = tau; out[f'i{{world}}'] = rep['iters']
np.savez({str(tmp_path / 'lv.npz')!r}, **out)
"""
    env = dict(os.environ, ACS_DIST_BACK_LEVELS='1')
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lv = np.load(tmp_path / 'lv.npz')
    for world in (3, 8):
        X, tau, rep = ours[world]
        assert rep['iters'] == int(lv[f'i{world}'])
        np.testing.assert_array_equal(X, lv[f'X{world}'])
        np.testing.assert_array_equal(tau, lv[f't{world}'])


def _rccl_worker(rank, world, port, out_dir):
    """One rank over the nccl (RCCL) backend, the configs[3] bench leg's exchange: a
    one-rank group on this single-GPU box (RCCL wants one device per rank), so every
    all-reduce of the frame-window protocol runs through RCCL on the device payloads."""
    import torch
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    tdist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', 0))
    try:
        ctx = _native.Context(0)
        prob, cams, X0 = _problem(40)
        table = pkin.build_table(prob.mode)
        t = torch.arange(4, dtype=torch.float64, device='cuda:0')
        tdist.all_reduce(t)
        X, tau, rep = dist.fte_solve_dist(ctx, table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
        np.savez(os.path.join(out_dir, f'rccl{rank}.npz'), X=X, tau=tau, iters=rep['iters'], t=t.cpu().numpy())
    finally:
        tdist.destroy_process_group()


def test_fte_dist_over_rccl_one_rank(ctx, tmp_path):
    """The RCCL exchange of the frame-window solve executes: a one-rank nccl process group
    (HSA_ENABLE_IPC_MODE_LEGACY=0 as exported on the box) runs dist.fte_solve_dist with every
    payload all-reduced by RCCL; the result is the single-GPU solve's."""
    import torch.multiprocessing as mp
    mp.start_processes(_rccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True, start_method='spawn')
    prob, cams, X0 = _problem(40)
    table = pkin.build_table(prob.mode)
    X1, t1, r1 = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0)
    a = np.load(tmp_path / 'rccl0.npz')
    np.testing.assert_array_equal(a['t'], np.arange(4.0))
    assert int(a['iters']) == r1['iters']
    np.testing.assert_allclose(a['X'], X1, rtol=0, atol=1e-9)
