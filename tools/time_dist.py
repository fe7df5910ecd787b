"""Frame-window FTE rounds on one GPU: wall time per solve and per round of the round
protocol (acinoset_amd.dist.lm_loop, one all-reduce per LM step) with 1 rank (the chain is
the whole trajectory) and 2 / 4 ranks emulated in one process on the same GPU (local sum
instead of RCCL), next to the single-GPU acs_fte_solve of the same problem.

    python tools/time_dist.py [frames ...] [--worlds 1,2,4]      (default 1000 10000; 1,2,4)

The emulated ranks run one after the other on one stream, so a round's time over the world
is the sum of the ranks' rounds: divided by the world it is the per-rank round an 8-GPU job
would spend (plus its RCCL all-reduce, which the local sum here replaces).
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acinoset_amd import _native, dist, workloads  # noqa: E402


def main():
    import torch
    argv = sys.argv[1:]
    worlds = (1, 2, 4)
    if '--worlds' in argv:
        i = argv.index('--worlds')
        worlds = tuple(int(w) for w in argv[i + 1].split(','))
        argv = argv[:i] + argv[i + 2:]
    frames = [int(a) for a in argv] or [1000, 10000]
    ctx = _native.Context(0)
    for N in frames:
        wl = workloads.fte_workload(ctx, N)
        args = (ctx, wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0)
        # single-GPU reference
        ctx.fte_solve(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0)
        t0 = time.perf_counter()
        X1, t1, r1 = ctx.fte_solve(wl.table, wl.cams, wl.meas, wl.w, wl.Ts, wl.qinv, wl.X0)
        ts = time.perf_counter() - t0
        print(f'N={N} acs_fte_solve: {ts * 1e3:.2f} ms, {r1["iters"]} iterations ({ts / r1["iters"] * 1e6:.0f} us each)',
              flush=True)
        dv = torch.device('cuda', 0)
        T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dv, dt)  # noqa: E731
        dev = dict(ints=T(wl.table.ints, torch.int32), reals=T(wl.table.reals), cams=T(wl.cams), meas=T(wl.meas),
                   w=T(wl.w), qinv=T(wl.qinv), X=T(wl.X0), tau=torch.zeros(len(wl.cams), dtype=torch.float64,
                                                                          device=dv))
        for world in worlds:
            with dist._on_torch_stream(ctx):
                for rep in range(3):
                    ranks = [dist.HipFteRank(*args, rank=r, world=world, dev=dev) for r in range(world)]
                    calls = []

                    def counting(p):
                        calls.append(1)
                        dist.local_allreduce(p)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    st = dist.lm_loop(ranks, counting)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    X, tau, info = ranks[0].result()
                    for r in ranks:
                        r.close()
                rounds = len(calls) - 2
                err = float(np.abs(X - X1).max())
                print(f'N={N} world={world} (emulated on 1 GPU): {dt * 1e3:.2f} ms per solve, status {st}, '
                      f'{info["iters"]} iterations, {rounds} rounds = all-reduces per solve {len(calls)} '
                      f'({dt / max(1, rounds) * 1e6:.0f} us per round for all {world} ranks, '
                      f'{dt / max(1, rounds) / world * 1e6:.0f} us per rank), '
                      f'max |X - single-GPU X| {err:.1e}', flush=True)


if __name__ == '__main__':
    main()
