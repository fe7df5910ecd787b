"""CPU tests of the frame-window distributed FTE protocol (acinoset_amd/dist.py, SURVEY.md
§8(e)): the product's LM driver `lm_loop` runs the oracle restatement of every rank
(oracle/fte_dist.py) and must reproduce the monolithic oracle solve (oracle/fte.py) —
single-process emulation for several rank counts, and world_size 2 over torch.distributed
with the gloo backend (the same all-reduce calls the GPU ranks make over RCCL).

Tolerance: the decomposition only reorders sums, so iterates agree to rounding: same
iteration count and status, cost 1e-12 relative, X 1e-10, tau 1e-12.
"""
import os
import socket

import numpy as np
import pytest

from acinoset_amd import dist, synth
from oracle import fte as ofte, fte_dist as odist


def _problem(mode='head', N=40, sd=True, inter='vel', seed=2):
    scene = synth.load_scene_file()
    seq = synth.make_sequence(N, scene, mode=mode, seed=seed, tau_max=0.004 if sd else 0.0)
    w = np.where(seq.likelihood > 0.5, 1.0 / 3.0, 0.0)
    prob = ofte.Problem(mode, seq.uv, w, scene.K, scene.D, scene.R, scene.t, seq.Ts, sd=sd, intermode=inter)
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
