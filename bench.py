#!/usr/bin/env python3
"""Benchmark of the MI355X SBA/FTE hot path (BASELINE.json metric:
"frames/sec to FTE/SBA convergence, 6-cam x 20-kp; reproj-px-RMS vs ref").

Default workload = BASELINE.json configs[1]: points-only SBA of a 6-camera, 100-frame,
20-keypoint synthetic sequence (12,000 observation slots, ~2,000 points) on one GPU.
One step = one full solve to convergence (reset of the initial points + the fused LM
kernel) with every input already resident in HBM. `value` = frames solved per second
over all ranks. Multi-GPU (torchrun): every rank solves its own frame shard (weak
scaling, no data-path collective: SBA points are independent).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8 TB/s HBM3E (spec)
FP64_PEAK_TFS = 78.6    # MI355X FP64 vector/matrix (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--frames', type=int, default=100, help='frames per rank (configs[1]: 100)')
    ap.add_argument('--cams', type=int, default=6)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--fte', action='store_true', help='also time the FTE trajectory solve (configs[2])')
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from acinoset_amd import _native, synth

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        # control plane only (barrier + max of the timed interval); the SBA data path
        # has no collective. gloo keeps RCCL out of a path that does not need it.
        dist.init_process_group('gloo')
    torch.cuda.set_device(local)
    ctx = _native.Context(local)
    # one explicit (non-null) stream carries the copies, the kernels and the timing events
    stream = torch.cuda.Stream(device=local)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # ---- workload: rank-local frame shard of a synthetic sequence --------------------
    scene = synth.load_scene_file() if args.cams == 6 else synth.ring_scene(args.cams)
    seq = synth.make_sequence(args.frames, scene, mode='default_nolure', seed=1000 * rank)
    uv, mask, pts0, truth, _ = synth.dense_sba_problem(seq)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    n_pts, C = mask.shape
    dev = torch.device('cuda', local)
    d_cams = torch.from_numpy(cams).to(dev)
    d_uv = torch.from_numpy(uv).to(dev)
    d_mask = torch.from_numpy(mask).to(dev)
    d_pts0 = torch.from_numpy(pts0).to(dev)
    d_pts = d_pts0.clone()
    opts = _native.Context.sba_opts()

    def step():
        d_pts.copy_(d_pts0, non_blocking=True)
        ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts,
                                 d_pts.data_ptr(), opts)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness + convergence of the same computation (untimed)
    d_pts.copy_(d_pts0)
    rep = ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts,
                                   d_pts.data_ptr(), opts, report=True)
    sol = d_pts.cpu().numpy()
    pos_rms = float(np.sqrt(np.mean(np.sum((sol - truth) ** 2, 1))))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        d_pts.copy_(d_pts0, non_blocking=True)
        ev[i][0].record(stream)
        ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts,
                                 d_pts.data_ptr(), opts)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = 1e3 * dt / args.steps
    frames_total = args.frames * world * args.steps
    value = frames_total / dt

    # roofline of the dominant kernel (k_sba_lm): algorithmic bytes per launch =
    # frames x B_SBA, B_SBA = C*L*(2*8 + 1) + 2*3*L*8; the fused kernel
    # streams the observation tensor once per solve, so this is also its HBM traffic floor.
    L = 20
    b_frame = C * L * 17 + 6 * L * 8
    bytes_launch = args.frames * b_frame
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    iters_mean = rep['iters_sum'] / max(1, rep['n_problems'])

    out = {
        'metric': 'frames/sec to SBA convergence, 6-cam x 20-kp (points-only SBA, configs[1])',
        'value': value,
        'unit': 'frames/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms_per_step,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic (acinoset_amd.synth: dummy_scene.json cameras, 1 px noise, 5% dropout, 1% outliers)',
        'config': {'workload': f'sba_points C={C} frames={args.frames}/rank L=20 (configs[1])',
                   'n_points_per_rank': int(n_pts), 'obs_slots_per_rank': int(n_pts * C),
                   'parallelism': f'frame-shard x{world}'},
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
                     'kernel': 'k_sba_lm', 'kernel_ms': kern_ms, 'bytes_per_launch': bytes_launch},
        'convergence': {'status': rep['status_counts'], 'iters_max': rep['iters_max'],
                        'gn_steps_mean': iters_mean, 'cost_before': rep['cost_before'],
                        'cost_after': rep['cost_after'], 'pos_rms_vs_truth_m': pos_rms},
    }

    if args.fte:
        out['fte'] = bench_fte(ctx, torch, stream)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(seq, scene, uv, mask, pts0, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(seq, scene, uv, mask, pts0, seconds):
    """Oracle (float64 numpy port of the per-point robust LM; 1 core) timed on a
    bounded sample of the same workload: repeated full solves for ~`seconds`."""
    from oracle import sba as osba
    n_pts, C = mask.shape
    pi, ci = np.nonzero(mask)
    p2 = uv[pi, ci]
    t0 = time.perf_counter()
    reps = 0
    while True:
        osba.sba_points(p2, pts0, pi, ci, scene.K, scene.D, scene.R, scene.t)
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {'value': reps * seq.N / dt, 'unit': 'frames/s', 'cores': 1, 'kind': 'port',
            'sample': f'{reps} full solves of the same {seq.N}-frame x {C}-cam x 20-kp problem '
                      f'(oracle/sba.py, numpy float64), {dt:.1f} s'}


def bench_fte(ctx, torch, stream):  # filled in by the FTE milestone
    return None


if __name__ == '__main__':
    main()
