"""CPU tests of the multi-GPU protocols (acinoset_amd/dist.py).

The product's LM driver (`lm_loop`, for the frame-window FTE and for points +
extrinsics SBA) run the oracle restatement of every rank (oracle/fte_dist.py,
oracle/sba_ext_dist.py) and must reproduce the monolithic oracle solves (oracle/fte.py,
oracle/sba_ext.py): single-process emulation for several rank counts, and world_size 2
over torch.distributed with the gloo backend (the same all-reduce calls the GPU ranks make
over RCCL).

Tolerance: the decompositions only reorder sums, so iterates agree to rounding: same
iteration count and status, cost 1e-12 relative, X 1e-10 (FTE) / 1e-9 (SBA), tau 1e-12.
"""
import os
import socket

import numpy as np
import pytest

from acinoset_amd import dist, synth
from oracle import fte as ofte, fte_dist as odist, sba_ext_dist as osed


def _problem(mode='head', N=40, sd=True, inter='vel', seed=2, sd_mode='const'):
    scene = synth.load_scene_file()
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed, tau_max=0.004 if sd else 0.0)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem(mode, seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=sd, intermode=inter,
                        sd_mode=sd_mode)
    X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
    return prob, X0


def _check(res, ref):
    Xd, taud, idd = res
    Xm, taum, im = ref
    assert idd['iters'] == im['iters'] and idd['n_accepted'] == im['n_accepted']
    assert {2: 'ftol', 3: 'xtol', 5: 'maxiter', 1: 'gtol', 4: 'stalled'}[idd['status']] == im['status']
    assert abs(idd['cost_after'] - im['cost_after']) <= 1e-12 * im['cost_after']
    np.testing.assert_allclose(Xd, Xm, rtol=0, atol=1e-10)
    np.testing.assert_allclose(taud, taum, rtol=0, atol=1e-12)


@pytest.mark.parametrize('mode,N,sd,inter', [('head', 40, True, 'vel'), ('head', 31, False, 'pos'),
                                             ('head', 20, True, 'acc'), ('head', 7, True, 'vel')])
@pytest.mark.parametrize('world', [2, 3, 8])
def test_dist_protocol_matches_monolithic(mode, N, sd, inter, world):
    prob, X0 = _problem(mode, N, sd, inter)
    ref = ofte.solve(prob, X0, max_iters=30)
    ranks = [odist.OracleFteRank(prob, X0, None, r, world, max_iters=30) for r in range(world)]
    dist.lm_loop(ranks, dist.local_allreduce)
    outs = [r.result() for r in ranks]
    for o in outs[1:]:                       # replicated state, bit for bit
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1], outs[0][1])
    _check(outs[0], ref)


@pytest.mark.parametrize('reject_at', [None, 3])
def test_dist_one_allreduce_per_lm_step(reject_at):
    """The round protocol: one all-reduce per LM step (init and the final gather aside),
    one more per rejected step, one more for the round queued before the stop was read.
    These problems never reject a step on their own, so `reject_at` inflates the 4th step's
    trial cost on every rank: the rejection, its re-formed round and the recovery run, and
    the solve still lands on the monolithic solution."""
    prob, X0 = _problem('head', 40, True, 'vel')
    world = 3
    ref = ofte.solve(prob, X0, max_iters=30)
    ranks = [odist.OracleFteRank(prob, X0, None, r, world, max_iters=30) for r in range(world)]
    if reject_at is not None:
        for r in ranks:
            def ph3(_orig=r.phase3, _r=r):
                p3 = _orig()
                if _r.iters == reject_at:
                    p3 = p3.copy()
                    p3[0] += 1e6 / world
                return p3
            r.phase3 = ph3
    sizes = []

    def counting(payloads):
        sizes.append(len(payloads[0]))
        dist.local_allreduce(payloads)
    dist.lm_loop(ranks, counting)
    X, tau, info = ranks[0].result()
    n_rej = info['iters'] - info['n_accepted']
    rounds = len(sizes) - 2                       # minus init and the final gather
    assert all(n == ranks[0].n1 + ranks[0].n3 for n in sizes[:-1])
    # round 0 forms step 1, round k decides step k and forms step k + 1 (a rejected step
    # adds the round that re-forms the system); plus the round queued before the stop was read
    assert rounds == info['iters'] + n_rej + 2, (rounds, info)
    if reject_at is None:
        _check((X, tau, info), ref)
    else:
        assert n_rej == 1 and info['status'] in (2, 3)
        np.testing.assert_allclose(X, ref[0], rtol=0, atol=1e-8)
        assert abs(info['cost_after'] - ref[2]['cost_after']) <= 1e-10 * ref[2]['cost_after']


@pytest.mark.parametrize('inter,N', [('vel', 24), ('acc', 17)])
@pytest.mark.parametrize('world', [2, 3, 8])
def test_dist_protocol_variable_delays_matches_monolithic(inter, N, world):
    """shutter_delay_mode='variable' (src/core/fte.py:238): every frame's delays are
    eliminated by the rank owning the frame; the solution rows and delays are gathered once."""
    prob, X0 = _problem('head', N, True, inter, sd_mode='variable')
    ref = ofte.solve(prob, X0, max_iters=30)
    ranks = [odist.OracleFteRank(prob, X0, None, r, world, max_iters=30) for r in range(world)]
    dist.lm_loop(ranks, dist.local_allreduce)
    outs = [r.result() for r in ranks]
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1], outs[0][1])
    assert outs[0][1].shape == (N, 6)
    _check(outs[0], ref)


def test_dist_chain_partition_covers_every_term():
    """Every frame and stencil is owned by exactly one rank; chains tile the blocks."""
    prob, X0 = _problem('head', 50)
    for world in (1, 2, 3, 4, 7, 8, 16):
        ranks = [odist.OracleFteRank(prob, X0, None, r, world) for r in range(world)]
        np.testing.assert_array_equal(sum(r.frames.astype(int) for r in ranks), 1)
        np.testing.assert_array_equal(sum(r.stencils.astype(int) for r in ranks), 1)
        published = np.concatenate([r.out for r in ranks])
        assert len(published) == len(set(published)) == prob.M * prob.P


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        prob, X0 = _problem('head', 40, True, 'vel')
        r = odist.OracleFteRank(prob, X0, None, rank, world, max_iters=30)
        allreduce = dist.torch_allreduce()

        def numpy_allreduce(payloads):   # gloo reduces the numpy buffers in place
            allreduce([torch.from_numpy(payloads[0])])
        dist.lm_loop([r], numpy_allreduce)
        X, tau, info = r.result()
        np.savez(os.path.join(out_dir, f'rank{rank}.npz'), X=X, tau=tau, iters=info['iters'],
                 nacc=info['n_accepted'], status=info['status'], cost=info['cost_after'])
    finally:
        tdist.destroy_process_group()


def test_dist_gloo_world2_matches_monolithic(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_gloo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method='spawn')
    prob, X0 = _problem('head', 40, True, 'vel')
    ref = ofte.solve(prob, X0, max_iters=30)
    res = [np.load(tmp_path / f'rank{r}.npz') for r in range(world)]
    assert np.array_equal(res[0]['X'], res[1]['X']) and np.array_equal(res[0]['tau'], res[1]['tau'])
    r0 = res[0]
    _check((r0['X'], r0['tau'], dict(iters=int(r0['iters']), n_accepted=int(r0['nacc']), status=int(r0['status']),
                                     cost_after=float(r0['cost']))), ref)


# ---- points + extrinsics SBA over ranks (acs_sba_ext_dist_*) ------------------------
def _ext_problem():
    from conftest import golden
    g = golden('sba_extrinsics')
    return g, g['points_2d'], g['points_3d'], g['point_indices'].astype(np.int64), g['camera_indices'].astype(np.int64)


def _ext_ranks(world, max_iters=200):
    g, uv, X, pi, ci = _ext_problem()
    ranks = []
    for r, (lo, hi, obs, loc) in enumerate(dist.split_points(pi, len(X), world)):
        ranks.append(osed.OracleSbaExtRank(uv[obs], X[lo:hi], loc, ci[obs], g['K'], g['D'], g['R0'], g['t0'], r, world,
                                           max_iters=max_iters))
    return ranks


def test_split_points_rejects_empty_shards():
    """More ranks than points, or a shard whose points have no observation: the same
    ValueError on every rank (each computes every shard) before any collective."""
    pi = np.array([0, 0, 1, 2, 2, 4], np.int64)   # point 3 unobserved
    assert [len(s[2]) for s in dist.split_points(pi, 5, 2)] == [3, 3]
    with pytest.raises(ValueError, match='each rank needs at least one'):
        dist.split_points(pi, 5, 8)
    with pytest.raises(ValueError, match='has no observation'):
        dist.split_points(pi, 5, 5)          # rank 3 holds point 3 only


@pytest.mark.parametrize('world', [2, 3, 7])
def test_ext_dist_protocol_matches_monolithic(world):
    from oracle import sba_ext as ose
    g, uv, X, pi, ci = _ext_problem()
    Xm, Rm, tm, im = ose.sba_extrinsics(uv, X, pi, ci, g['K'], g['D'], g['R0'], g['t0'], max_iters=200)
    ranks = _ext_ranks(world)
    sizes = []

    def counting(payloads):
        sizes.append(len(payloads[0]))
        dist.local_allreduce(payloads)
    dist.lm_loop(ranks, counting)
    outs = [r.result() for r in ranks]
    # one all-reduce per LM step: init, one round per step (+1 per rejected step), and the
    # round queued before the stop was read
    n_rej = outs[0][3]['iters'] - outs[0][3]['n_accepted']
    assert len(sizes) - 1 == outs[0][3]['iters'] + n_rej + 2, (len(sizes), outs[0][3])
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1], outs[0][1])
    R, t, _, info = outs[0]
    Xd = np.concatenate([o[2] for o in outs])
    assert info['iters'] == im['iters'] and info['n_accepted'] == im['n_accepted']
    assert {2: 'ftol', 3: 'xtol', 5: 'maxiter'}[info['status']] == im['status']
    assert abs(info['cost_after'] - im['cost_after']) <= 1e-12 * im['cost_after']
    np.testing.assert_allclose(Xd, Xm, rtol=0, atol=1e-9)
    np.testing.assert_allclose(R, Rm, rtol=0, atol=1e-10)
    np.testing.assert_allclose(t, tm, rtol=0, atol=1e-9)


def test_dist_max_iters_zero_takes_no_step():
    """max_iters = 0: no LM step on any rank, as the monolithic solve (X0 back, iters 0,
    status 'maxiter') - the first round stops before stepping (frame-window FTE and
    points + extrinsics SBA)."""
    prob, X0 = _problem('head', 20, True, 'vel')
    ref = ofte.solve(prob, X0, max_iters=0)
    assert ref[2]['iters'] == 0 and np.array_equal(ref[0], X0)
    ranks = [odist.OracleFteRank(prob, X0, None, r, 2, max_iters=0) for r in range(2)]
    assert dist.lm_loop(ranks, dist.local_allreduce) == 5
    Xd, taud, info = ranks[0].result()
    assert info['iters'] == 0 and info['n_accepted'] == 0
    np.testing.assert_array_equal(Xd, X0)
    ranks = _ext_ranks(2, max_iters=0)
    assert dist.lm_loop(ranks, dist.local_allreduce) == 5
    g, uv, X, pi, ci = _ext_problem()
    R, t, Xr, info = ranks[0].result()
    assert info['iters'] == 0
    np.testing.assert_array_equal(np.concatenate([r.result()[2] for r in ranks]), X)


def _gloo_ext_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        r = _ext_ranks(world)[rank]
        allreduce = dist.torch_allreduce()
        dist.lm_loop([r], lambda ps: allreduce([torch.from_numpy(ps[0])]))
        R, t, X, info = r.result()
        np.savez(os.path.join(out_dir, f'ext{rank}.npz'), R=R, t=t, X=X, iters=info['iters'])
    finally:
        tdist.destroy_process_group()


def test_ext_dist_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    from oracle import sba_ext as ose
    mp.start_processes(_gloo_ext_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method='spawn')
    g, uv, X, pi, ci = _ext_problem()
    Xm, Rm, tm, im = ose.sba_extrinsics(uv, X, pi, ci, g['K'], g['D'], g['R0'], g['t0'], max_iters=200)
    a, b = (np.load(tmp_path / f'ext{r}.npz') for r in range(2))
    assert np.array_equal(a['R'], b['R']) and np.array_equal(a['t'], b['t'])
    assert int(a['iters']) == im['iters']
    np.testing.assert_allclose(np.concatenate([a['X'], b['X']]), Xm, rtol=0, atol=1e-9)
    np.testing.assert_allclose(a['R'], Rm, rtol=0, atol=1e-10)
