#!/usr/bin/env python3
"""Benchmark of the MI355X SBA/FTE hot path (BASELINE.json metric:
"frames/sec to FTE/SBA convergence, 6-cam x 20-kp; reproj-px-RMS vs ref").

Default workload = BASELINE.json configs[1]: points-only SBA of the 6-camera, 100-frame,
20-keypoint problem exactly as the reference built it (tests/golden/sba_cfg2.npz: the
reference's `_sba_points` run on synthetic observations - 2,000 points, 11,401
observations, its triangulated start) on one GPU. One step = one full solve to
convergence (the fused LM kernel reads the resident initial points and writes the
solution to a second buffer) with every input already in HBM. `value` = frames solved
per second over all ranks. The line also carries the metric's second half: the
reprojection RMS of the GPU solution next to the reference's (and the oracle's).
Multi-GPU (torchrun): every rank solves its own copy (weak scaling, no data-path
collective: SBA points are independent).

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
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--fte', action='store_true', default=True, help='also time the FTE solve (configs[2])')
    ap.add_argument('--no-fte', dest='fte', action='store_false')
    ap.add_argument('--window-frames', type=int, default=10000,
                    help='configs[3]: FTE over this many frames, frame windows sharded over the ranks (0 = skip)')
    ap.add_argument('--ekf-seqs', type=int, default=64, help='EKF + RTS leg: sequences per rank (0 = skip)')
    ap.add_argument('--ekf-frames', type=int, default=500)
    ap.add_argument('--ekf-cams', type=int, default=12)
    ap.add_argument('--pipeline-seqs', type=int, default=80,
                    help='configs[4] fused SBA+EKF leg: clips per rank (0 = skip)')
    ap.add_argument('--pipeline-frames', type=int, default=250)
    ap.add_argument('--exchange', default='nccl', choices=('nccl', 'gloo'),
                    help='backend of the FTE window all-reduces (nccl = RCCL over xGMI)')
    ap.add_argument('--scale-frames', type=int, default=20000,
                    help='also time SBA at configs[4] scale on one GPU (0 = skip)')
    ap.add_argument('--scale-cams', type=int, default=12)
    ap.add_argument('--fte-frames', type=int, default=1000)
    ap.add_argument('--no-graph', dest='graph', action='store_false', default=True,
                    help='launch the K timed solves one by one on the stream instead of replaying them '
                         'from one captured hipGraph')
    ap.add_argument('--event-every', type=int, default=8,
                    help='HIP event pairs bracket groups of this many consecutive timed steps '
                         '(kernel duration for the roofline)')
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
    # one GPU per rank; wrapping onto fewer devices only happens in a rehearsal on a
    # single-GPU box (torchrun --nproc-per-node 2 ... --exchange gloo)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    ctx = _native.Context(local)
    # one explicit (non-null) stream carries the copies, the kernels and the timing events
    stream = torch.cuda.Stream(device=local)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # ---- workload: the reference's own configs[1] SBA problem (every rank solves its own
    # copy: weak scaling, SBA points are independent, no data-path collective) -----------
    from acinoset_amd import workloads
    wl = workloads.sba_reference_workload()
    uv, mask, pts0, cams = wl.uv, wl.mask, wl.pts0, wl.cams
    n_pts, C = mask.shape
    dev = torch.device('cuda', local)
    # raw device pointers go to the C ABI: contiguous device copies
    d_cams, d_uv, d_mask, d_pts0 = (torch.from_numpy(np.ascontiguousarray(a)).to(dev).contiguous()
                                    for a in (cams, uv, mask, pts0))
    d_pts = d_pts0.clone()
    opts = _native.Context.sba_opts()

    # one step = one full solve from the resident initial points (pts_in -> pts_out): a direct
    # call of the C ABI entry acs_sba_points_dense_io with pre-marshalled device pointers
    import ctypes
    fn = ctx.lib.acs_sba_points_dense_io
    call = (ctx.h, ctypes.c_void_p(d_cams.data_ptr()), C, ctypes.c_void_p(d_uv.data_ptr()),
            ctypes.c_void_p(d_mask.data_ptr()), n_pts, ctypes.c_void_p(d_pts0.data_ptr()),
            ctypes.c_void_p(d_pts.data_ptr()), ctypes.byref(opts), None, _native.ACS_DEVICE_PTRS)

    def step():
        rc = fn(*call)
        if rc:
            ctx.check(rc, 'acs_sba_points_dense_io')

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness + convergence of the same computation (untimed)
    rep = ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts,
                                   d_pts.data_ptr(), opts, report=True, pts_in_p=d_pts0.data_ptr())
    sol = d_pts.cpu().numpy()
    pos_rms = float(np.sqrt(np.mean(np.sum((sol - wl.truth) ** 2, 1))))
    # the metric's second half (untimed): reprojection RMS of the GPU solution against the
    # reference's own solution of the same problem (its residuals['after'])
    res_gpu = ctx.sba_residuals(cams, wl.points_2d, wl.point_idx, wl.cam_idx, sol)
    rms_gpu, rms_ref = workloads.reproj_rms(res_gpu), workloads.reproj_rms(wl.ref_resid_after)
    dref = np.sqrt(np.sum((sol - wl.ref_pts) ** 2, 1))

    # HIP events on the kernel's stream bracket consecutive groups of `every` steps (a pair
    # per launch would cost more host time than the launch itself and add its own latency
    # to the bracket); kernel_ms = bracketed GPU time / launches
    every = max(1, min(args.event_every, args.steps))
    ngrp = args.steps // every

    def timed_stream():
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(ngrp)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            g, j = divmod(i, every)
            if g < ngrp and j == 0:
                ev[g][0].record(stream)
            step()
            if g < ngrp and j == every - 1:
                ev[g][1].record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0, float(np.mean([a.elapsed_time(b) for a, b in ev])) / every

    graph = None
    if args.graph:
        # the K timed solves captured once as K kernel nodes of one hipGraph (a graph node
        # costs ~1.6 us of dispatch, a stream launch ~2.5 us: profiles/r02/launch_probe.log);
        # every node is the full LM solve from the resident initial points. Captured and
        # replayed once before the timed region (untimed warm-up).
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for _ in range(args.steps):
                step()
        graph.replay()
        torch.cuda.synchronize()

    def timed_graph():
        # the host bracket holds the replay and the synchronisation only; the GPU clock (for
        # roofline.achieved) comes from a second replay bracketed by events. (Round 4 recorded
        # the start event outside the bracket and the end event inside it: asymmetric, ADVICE
        # r04; since round 5 neither is inside.)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        graph.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        return dt, e0.elapsed_time(e1) / args.steps

    def max_over_ranks(dt):
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    dt, kern_ms = timed_graph() if graph is not None else timed_stream()
    dt = max_over_ranks(dt)
    stream_line = None
    if graph is not None:
        # the same K solves launched one by one, for comparison (after the headline timing)
        dts, kms = timed_stream()
        dts = max_over_ranks(dts)
        stream_line = {'value': wl.n_frames * world * args.steps / dts, 'ms_per_step': 1e3 * dts / args.steps,
                       'kernel_ms': kms}
    ms_per_step = 1e3 * dt / args.steps
    frames_total = wl.n_frames * world * args.steps
    value = frames_total / dt

    # roofline of the dominant kernel (k_sba_lm): algorithmic bytes per launch =
    # frames x B_SBA, B_SBA = C*L*(2*8 + 1) + 2*3*L*8; the fused kernel
    # streams the observation tensor once per solve, so this is also its HBM traffic floor.
    L = 20
    b_frame = C * L * 17 + 6 * L * 8
    bytes_launch = wl.n_frames * b_frame
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    iters_mean = rep['iters_sum'] / max(1, rep['n_problems'])
    traffic, pmc = pmc_per_launch('k_sba_lm', n_pts * _lm_group(C, n_pts))

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
        'data': 'synthetic: the reference\'s own configs[1] run (tests/golden/sba_cfg2.npz: acinoset_amd.synth seed 0 '
                'on dummy_scene.json, 1 px noise, 5% dropout, 1% outliers; the reference\'s pairwise-triangulation '
                'start and point selection)',
        'config': {'workload': f'sba_points C={C} frames={wl.n_frames}/rank L=20 (configs[1])',
                   'n_points_per_rank': int(n_pts), 'obs_slots_per_rank': int(n_pts * C),
                   'parallelism': f'frame-shard x{world}'},
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                     'kernel': 'k_sba_lm', 'kernel_ms': kern_ms,
                     'kernel_ms_launches': args.steps if graph is not None else ngrp * every,
                     'bytes_per_launch': bytes_launch,
                     'traffic_source': pmc['source'] if pmc else None,
                     'note': f'latency-bound at this size: {int(n_pts * _group(C) // 64)} waves for '
                             f'{4 * 256} SIMDs, each a chain of up to {rep["iters_max"]} dependent LM iterations '
                             '(~1.25 us each, profiles/r02/sba_iters.log) after a 2.4 us stream-launch floor; '
                             'sba_at_scale carries the throughput rooflines'},
        'convergence': {'status': rep['status_counts'], 'iters_max': rep['iters_max'],
                        'gn_steps_mean': iters_mean, 'cost_before': rep['cost_before'],
                        'cost_after': rep['cost_after'], 'pos_rms_vs_truth_m': pos_rms},
        'launch': ('one hipGraph of the K solves (K kernel nodes), replayed once in the timed region'
                   if graph is not None else 'K stream launches'),
        'stream_launch': stream_line,
        'reproj_rms_px': rms_gpu,
        'reproj_rms_ref_px': rms_ref,
        'reproj_rms_vs_ref_px': rms_gpu - rms_ref,
        'pos_vs_ref_m': {'rms': float(np.sqrt(np.mean(dref ** 2))), 'max': float(dref.max()),
                         'note': 'against the reference\'s scipy TRF solution of the same problem '
                                 '(it stops on xtol; SURVEY.md §8(a) a4)'},
    }
    out['roofline_fp64'] = sba_fp64_roofline(int(mask.sum()), n_pts, iters_mean, kern_ms, pmc)
    if pmc and pmc.get('valu_insts') and pmc.get('waves'):
        # the issue rate of one wave: VALU instructions per wave (PMC) over the kernel's time
        # in 2.4 GHz clocks
        ipw = pmc['valu_insts'] / pmc['waves']
        out['roofline_fp64'].update({
            'valu_insts_per_wave': ipw, 'clocks_per_valu_inst': kern_ms * 1e-3 * 2.4e9 / ipw,
            'note': 'one wave per busy SIMD: each wave issues its VALU stream serially, so time ~ '
                    'instructions per wave x issue interval (f64 FMA: 8 clocks dependent latency, '
                    'profiles/r01d/probes)'})

    def leg(name, fn):
        # a side leg reports its failure in the line instead of costing the headline
        try:
            out[name] = fn()
        except Exception as e:  # noqa: BLE001
            out[name] = {'error': f'{type(e).__name__}: {e}'}

    if args.fte and world == 1:
        leg('fte', lambda: bench_fte(ctx, torch, stream, n_frames=args.fte_frames, cpu=not args.no_cpu_baseline))
    if args.ekf_seqs > 0:
        # the EKF throughput is quoted on the model that tracks these sequences ('head');
        # the reference's 29-parameter 'default' model loses them within ~20 frames (as its
        # own golden run does, tests/golden/ekf_default.npz), so that leg is labelled and
        # kept only as a cost figure for the bigger state
        leg('ekf', lambda: bench_ekf(ctx, torch, args.ekf_seqs, args.ekf_frames, args.ekf_cams, world, rank,
                                     mode='head'))
        leg('ekf_analytic_h', lambda: bench_ekf(ctx, torch, args.ekf_seqs, args.ekf_frames, args.ekf_cams, world,
                                                rank, mode='head', jacobian='analytic'))
        leg('ekf_default_model_diverges', lambda: bench_ekf(ctx, torch, args.ekf_seqs, args.ekf_frames,
                                                            args.ekf_cams, world, rank, mode='default'))
    if args.pipeline_seqs > 0:
        leg('sba_ekf_pipeline', lambda: bench_pipeline(ctx, torch, stream, world, rank, args.pipeline_seqs,
                                                       args.pipeline_frames))
    if args.window_frames > 0:
        leg('fte_window', lambda: bench_fte_window(ctx, torch, stream, args.window_frames, world, rank,
                                                   args.exchange))
    if args.scale_frames > 0 and world == 1:
        leg('sba_at_scale', lambda: bench_sba_scale(ctx, torch, stream, args.scale_frames, args.scale_cams))

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'], sol_o = cpu_baseline(wl, args.cpu_seconds)
        res_o = ctx.sba_residuals(cams, wl.points_2d, wl.point_idx, wl.cam_idx, sol_o)
        do = np.sqrt(np.sum((sol - sol_o) ** 2, 1))
        out['reproj_rms_oracle_px'] = workloads.reproj_rms(res_o)
        out['reproj_rms_vs_oracle_px'] = rms_gpu - out['reproj_rms_oracle_px']
        out['pos_vs_oracle_m'] = {'rms': float(np.sqrt(np.mean(do ** 2))), 'max': float(do.max())}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


FP64_VALU_PEAK_TFS = 78.6  # MI355X FP64 vector peak (spec sheet)


def pmc_per_launch(kernel, grid):
    """HBM bytes / FP64 flops per launch of `kernel` at `grid` threads from the newest
    committed PMC summary (profiles/r*/traffic.json, tools/pmc_summary.py: separate
    FETCH_SIZE (x2, gfx950) and WRITE_SIZE passes of this bench). None if not profiled."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r*',
                                          'traffic.json')))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    r = d['per_launch'].get(f'{kernel}@{grid}')
    if r is None:
        return None, None
    root = os.path.dirname(os.path.abspath(__file__))
    c = r.get('counters', {})
    return r.get('hbm_bytes'), dict(fp64_flops=r.get('fp64_flops'), valu_insts=r.get('valu_insts'),
                                    waves=c.get('SQ_WAVES'), source=os.path.relpath(files[-1], root))


def _group(C):
    g = 2
    while g < C:
        g *= 2
    return g


def _lm_group(K, n_pts, n_cu=256):
    """Lanes per point of k_sba_lm as run_lm (sba.hip) picks them: nextpow2(K), or in a
    throughput-bound grid (> 16 waves per CU) groups of three slots per lane where that wastes
    fewer lanes (K = 12: 4 lanes) - the PMC summary is keyed by the launch's thread count."""
    g = _group(K)
    if g > 64:
        return 64
    if g > K and (n_pts * g + 63) // 64 > 16 * n_cu:
        g3 = _group((K + 2) // 3) if (K + 2) // 3 > 1 else 1
        if 3 * g3 < g:
            return max(g3, 2)
    return g


def host_cpu():
    """(model name, usable cores): the cores this process may run on, capped by the
    harness's per-GPU CPU share (OMP_NUM_THREADS, 16 on the GPU box) when it is set."""
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get('OMP_NUM_THREADS')
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return model, max(1, n)


def _sba_oracle_worker(args):
    """One host core: repeated full oracle solves of the problem for ~`seconds`."""
    p2, pts0, pi, ci, K, D, R, t, seconds = args
    from oracle import sba as osba
    t0 = time.perf_counter()
    reps = 0
    sol = None
    while True:
        sol = osba.sba_points(p2, pts0, pi, ci, K, D, R, t)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps, dt, sol


def cpu_baseline(wl, seconds):
    """Oracle (float64 numpy port of the per-point robust LM, oracle/sba.py) timed on the
    host cores on a bounded sample of the same workload: every worker process (one per
    usable core, BLAS single-threaded) repeats full solves of the configs[1] problem for
    ~`seconds`; frames/s = sum over workers of solves x frames / own wall time. Returns
    (baseline dict, the oracle's solution)."""
    import multiprocessing as mp
    model, cores = host_cpu()
    job = (wl.points_2d, wl.pts0, wl.point_idx, wl.cam_idx, wl.K, wl.D, wl.R, wl.t, seconds)
    keep = {k: os.environ.get(k) for k in ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS')}
    try:
        for k in keep:
            os.environ[k] = '1'          # inherited by the spawned workers before numpy loads
        with mp.get_context('spawn').Pool(cores) as pool:
            res = pool.map(_sba_oracle_worker, [job] * cores)
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    value = sum(r * wl.n_frames / dt for r, dt, _ in res)
    reps = sum(r for r, _, _ in res)
    return ({'value': value, 'unit': 'frames/s', 'cores': cores, 'cpu_model': model,
             'nproc': os.cpu_count(), 'kind': 'port',
             'sample': f'{reps} full solves of the same {wl.n_frames}-frame x {wl.cam_idx.max() + 1}-cam x 20-kp '
                       f'problem (oracle/sba.py, numpy float64) on {cores} worker processes, ~{seconds:.0f} s each'},
            res[0][2])


def sba_fp64_roofline(n_obs, n_pts, gn_steps_mean, kern_ms, pmc):
    """k_sba_lm against the FP64 vector peak with ALGORITHMIC flops (150 flop
    per observation + 40 per point for one residual + Jacobian + GN evaluation), times the
    evaluations of a solve (the GN steps + the initial one), over the kernel's time. The PMC
    lane-flop count (64 x the f64 VALU instructions, FMA twice: what the kernel issues,
    including the null-camera lanes and the transcendental expansions) is kept beside it as
    issued_flops."""
    evals = gn_steps_mean + 1.0
    alg = (150.0 * n_obs + 40.0 * n_pts) * evals
    tfs = alg / (kern_ms * 1e-3) / 1e12
    r = {'bound': 'fp64-valu', 'achieved': tfs, 'peak': FP64_VALU_PEAK_TFS, 'unit': 'TFLOP/s',
         'frac': tfs / FP64_VALU_PEAK_TFS, 'flops_per_launch': alg, 'evaluations_per_solve': evals,
         'flop_model': '150/obs + 40/pt per evaluation (SURVEY.md 8(d))'}
    if pmc and pmc.get('fp64_flops'):
        itf = pmc['fp64_flops'] / (kern_ms * 1e-3) / 1e12
        r.update({'issued_flops_per_launch': pmc['fp64_flops'], 'issued_achieved': itf,
                  'issued_frac': itf / FP64_VALU_PEAK_TFS, 'issued_source': pmc['source']})
    return r


def bench_sba_scale(ctx, torch, stream, n_frames=20000, n_cams=12, steps=10):
    """configs[4] shape on one GPU (report the roofline fraction where the
    observation tensor is ~100 MB): 12-camera ring, 20,000 frames x 20 keypoints."""
    from acinoset_amd import _native, synth
    scene = synth.ring_scene(n_cams)
    seq = synth.make_sequence(n_frames, scene, mode='default_nolure', seed=4242)
    uv, mask, pts0, truth, _ = synth.dense_sba_problem(seq)
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    n_pts, C = mask.shape
    dev = torch.device('cuda', torch.cuda.current_device())
    d_cams = torch.from_numpy(cams).to(dev)
    d_uv = torch.from_numpy(uv).to(dev)
    d_mask = torch.from_numpy(mask).to(dev)
    d_pts0 = torch.from_numpy(pts0).to(dev)
    d_pts = d_pts0.clone()
    opts = _native.Context.sba_opts()
    def step():
        ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts, d_pts.data_ptr(),
                                 opts, pts_in_p=d_pts0.data_ptr())
    for _ in range(2):
        step()
    rep = ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts,
                                   d_pts.data_ptr(), opts, report=True, pts_in_p=d_pts0.data_ptr())
    pos_rms = float(np.sqrt(np.mean(np.sum((d_pts.cpu().numpy() - truth) ** 2, 1))))
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    L = 20
    bytes_launch = n_frames * (C * L * 17 + 6 * L * 8)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic, pmc = pmc_per_launch('k_sba_lm', n_pts * _lm_group(C, n_pts))
    fp64 = sba_fp64_roofline(int(mask.sum()), n_pts, rep['iters_sum'] / max(1, rep['n_problems']), kern_ms, pmc)
    return {'workload': f'sba_points C={C} frames={n_frames} L={L} (configs[4] shape, 1 GPU)',
            'frames_per_s': n_frames / dt, 'ms_per_step': dt * 1e3, 'n_points': int(n_pts),
            'obs': int(mask.sum()),
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'kernel': 'k_sba_lm', 'kernel_ms': kern_ms,
                         'bytes_per_launch': bytes_launch, 'traffic': traffic},
            'roofline_fp64': fp64,
            'iters_max': rep['iters_max'], 'gn_steps_mean': rep['iters_sum'] / max(1, rep['n_problems']),
            'status': rep['status_counts'], 'pos_rms_vs_truth_m': pos_rms}


def _fte_problem(ctx, n_frames, seed=77):
    """Synthetic FTE input (acinoset_amd.workloads, shared with the parity tests)."""
    from acinoset_amd import workloads
    wl = workloads.fte_workload(ctx, n_frames, seed=seed)
    return wl.seq, wl.cams, wl.meas, wl.w, wl.X0, wl.table, wl.qinv


def bench_ekf(ctx, torch, n_seq, n_frames, n_cams, world, rank, mode='default', steps=2, jacobian='fd'):
    """EKF + RTS smoother (the EKF half of configs[4]): `n_seq`
    independent synthetic sequences per rank (replicas: the filter is sequential in time),
    `n_cams`-camera ring, reference numerics. Reports the smoothed keypoints' RMS error
    against the synthetic truth and whether the filter tracks: the reference's 'default'
    model (29 pose parameters, 21 markers) diverges on these sequences within ~20 frames
    (its own golden run does too, tests/golden/ekf_default.npz; tools/ekf_tracking.py),
    the 'head' model (6 parameters, 3 markers) tracks to a few mm."""
    import importlib
    import torch.distributed as tdist
    from acinoset_amd import _native, synth
    from acinoset_amd.kinematics import build_table
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    scene = synth.load_scene_file() if n_cams == 6 else synth.ring_scene(n_cams)
    seqs = [synth.make_sequence(n_frames, scene, mode=mode, seed=500 + 97 * rank + k) for k in range(n_seq)]
    table = build_table(mode)
    P = table.P
    cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
    meas = np.stack([q.uv for q in seqs])
    lik = np.stack([q.likelihood for q in seqs])
    s0 = np.zeros((n_seq, 3 * P))   # first frame's pose and velocity (throughput leg, not an init study)
    for k, q in enumerate(seqs):
        s0[k, :P] = q.x[0]
        s0[k, P:2 * P] = (q.x[1] - q.x[0]) / q.Ts
    covs = cekf.ring_cal_covs(n_cams)
    args = (90.0, 0.5, float(scene.res[0]), cekf.measurement_std(n_cams, covs), cekf.process_covariance(P, 1 / 90.0),
            cekf.initial_covariance(mode))
    kw = dict(ref_numerics=jacobian == 'fd', jacobian=jacobian)
    out = ctx.ekf_run(table, cams, meas, lik, *args, s0, **kw)          # warm-up, and the outputs checked below
    # the timed calls: every input resident in HBM and the states written there (ACS_DEVICE_PTRS,
    # no host copy in the timed region; round 4 timed host arrays, ~24 % of a call was copies)
    dev = torch.device('cuda', torch.cuda.current_device())
    tens = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt).contiguous()  # noqa
    d_ints, d_reals = tens(table.ints, torch.int32), tens(table.reals)
    d_in = [tens(a) for a in (cams, meas, lik, args[3], args[4], args[5], s0)]
    n = 3 * P
    d_xe = torch.empty((n_seq, n_frames, n), dtype=torch.float64, device=dev)
    d_xs = torch.empty_like(d_xe)
    stream = torch.cuda.current_stream()

    def call():
        ctx.ekf_run_dev(d_ints.data_ptr(), d_ints.numel(), d_reals.data_ptr(), d_reals.numel(), d_in[0].data_ptr(),
                        n_cams, d_in[1].data_ptr(), d_in[2].data_ptr(), n_seq, n_frames, args[0], args[1], args[2],
                        d_in[3].data_ptr(), d_in[4].data_ptr(), d_in[5].data_ptr(), d_in[6].data_ptr(),
                        d_xe.data_ptr(), d_xs.data_ptr(), **kw)
    call()
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        call()
    e1.record(stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    gpu_ms = e0.elapsed_time(e1) / steps
    assert np.array_equal(d_xs.cpu().numpy(), out['x_smooth']), 'device-resident EKF differs from the host-array call'
    # the device-pointer calls do not check for singular solves themselves (asynchronous):
    # read the last call's counter after the timed region
    singular = ctx.ekf_singular_count()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    # smoothed keypoints vs the synthetic truth (first 4 sequences, untimed)
    errs = []
    for k in range(min(4, n_seq)):
        pe = ctx.fk(table, np.ascontiguousarray(out['x_smooth'][k][:, :P]))
        pt = ctx.fk(table, seqs[k].x)
        errs.append(np.sqrt(np.mean(np.sum((pe - pt) ** 2, -1))))
    rms = float(np.median(errs))
    L = table.L
    return {'workload': f'ekf+rts C={n_cams} {mode} (P={P}, L={L}) {n_seq} seqs x {n_frames} frames/rank',
            'frames_per_s': world * n_seq * n_frames / dt, 'ms_per_call': dt * 1e3, 'gpu_ms_per_call': gpu_ms,
            'inputs': 'device-resident (ACS_DEVICE_PTRS)',
            'us_per_frame_per_seq': dt / n_frames * 1e6, 'scaling': 'weak (replicas)',
            'smoothed_rms_vs_truth_m': rms, 'filter': 'tracks' if rms < 0.05 else 'diverged',
            'singular_solves_last_call': singular,
            'outliers_frac': float(np.mean(out['outliers'])) / max(1.0, float(np.sum(lik > 0.5)) * 2 / n_seq),
            'numerics': ('reference (float32 state rounding, FD Jacobian eps 1e-3)' if jacobian == 'fd' else
                         'float64, analytic H from the FK Jacobian (SURVEY §8(f)2)'),
            'kernel': 'k_ekf_filter_w1 (4 waves per sequence)' if P == 6 else 'k_ekf_filter (8 waves per sequence)'}


def bench_pipeline(ctx, torch, stream, world, rank, n_seq=80, n_frames=250, n_cams=12, steps=3):
    """configs[4]: "12-cam 20k-frame synthetic SBA+EKF fused" - per rank n_seq clips of n_frames
    frames (80 x 250 = 20,000 frames, ~2.8 s clips at 90 fps) on the synthesised 12-camera ring,
    20 DLC keypoints per frame. One step = acs_sba_ekf_pipeline on the HBM-resident observation
    tensor: pairwise triangulation + points-only SBA of every keypoint (core.sba), the EKF initial
    state fitted on the pairwise-triangulated points as core.ekf does (src/core/ekf.py:121-157;
    from_sba=False, the reference's semantics), and the EKF + RTS smoother (core.ekf) with the head model on
    its three markers (the 29-parameter 'default' model loses these sequences; see the ekf legs).
    Weak scaling: every rank runs its own clips (the EKF is sequential in time; clips are the
    parallel unit, no collective)."""
    import importlib
    import torch.distributed as tdist
    from acinoset_amd import _native, synth
    from acinoset_amd.kinematics import build_table
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    scene = synth.ring_scene(n_cams)
    seqs = [synth.make_sequence(n_frames, scene, mode='default_nolure', seed=3000 + 131 * rank + k)
            for k in range(n_seq)]
    obs_markers = seqs[0].markers
    table = build_table('head')
    P = table.P
    covs = cekf.ring_cal_covs(n_cams)
    dv = torch.device('cuda', torch.cuda.current_device())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dv).contiguous()  # noqa: E731
    d_cams = T(_native.pack_cameras(scene.K, scene.D, scene.R, scene.t))
    d_meas = T(np.stack([q.uv for q in seqs]))
    d_lik = T(np.stack([q.likelihood for q in seqs]))
    d_rstd = T(cekf.measurement_std(n_cams, covs))
    d_Q = T(cekf.process_covariance(P, 1 / 90.0))
    d_P0 = T(cekf.initial_covariance('head'))
    L = len(obs_markers)
    d_pts = torch.empty((n_seq, n_frames, L, 3), dtype=torch.float64, device=dv)
    d_xe = torch.empty((n_seq, n_frames, 3 * P), dtype=torch.float64, device=dv)
    d_xs = torch.empty_like(d_xe)
    args = (table, obs_markers, d_cams.data_ptr(), n_cams, d_meas.data_ptr(), d_lik.data_ptr(), n_seq, n_frames,
            90.0, 0.5, float(scene.res[0]), d_rstd.data_ptr(), d_Q.data_ptr(), d_P0.data_ptr(), d_pts.data_ptr(),
            d_xe.data_ptr(), d_xs.data_ptr())
    rep, outl = ctx.sba_ekf_pipeline_dev(*args, report=True)          # warm-up + convergence report
    torch.cuda.synchronize()
    pts = d_pts.cpu().numpy()
    xs = d_xs.cpu().numpy()
    truth = np.stack([q.pos3d[:, 0] for q in seqs])                   # (S, N, L, 3)
    ok = np.isfinite(pts).all(-1)
    sba_rms = float(np.sqrt(np.mean(np.sum((pts[ok] - truth[ok]) ** 2, -1))))
    head_err = []
    for k in range(min(8, n_seq)):
        pe = ctx.fk(table, np.ascontiguousarray(xs[k][:, :P]))
        head_err.append(np.sqrt(np.mean(np.sum((pe - truth[k][:, :3]) ** 2, -1))))
    if world > 1:
        tdist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        ctx.sba_ekf_pipeline_dev(*args)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    dt = (time.perf_counter() - t0) / steps
    gpu_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    frames = n_seq * n_frames
    # algorithmic HBM bytes per frame of the fused pass: the observation tensor read once
    # (pixels 16 B + likelihood 8 B per camera and keypoint), the SBA points and the filtered
    # and smoothed EKF states written once
    b_frame = n_cams * L * 24 + L * 3 * 8 + 2 * 3 * P * 8
    achieved = frames * b_frame / (gpu_ms * 1e-3) / 1e9
    return {'workload': f'sba+ekf fused C={n_cams} L={L} (EKF head model P={P}) {n_seq} clips x {n_frames} frames/rank '
                        f'(configs[4])',
            'frames_per_s': world * frames / dt, 'ms_per_step': dt * 1e3, 'gpu_ms_per_step': gpu_ms,
            'scaling': 'weak (clips per rank)',
            'sba': {'status': rep['status_counts'], 'iters_max': rep['iters_max'], 'points': int(rep['n_problems']),
                    'pos_rms_vs_truth_m': sba_rms},
            'ekf': {'smoothed_head_rms_vs_truth_m': float(np.median(head_err)),
                    'filter': 'tracks' if np.median(head_err) < 0.05 else 'diverged',
                    'outliers_per_clip': float(np.mean(outl))},
            'roofline': {'bound': 'latency (sequential EKF frames per clip)', 'achieved': achieved,
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                         'bytes_per_frame': b_frame,
                         'note': 'HBM-equivalent rate of the whole fused step; the EKF walks each clip\'s frames in '
                                 'order on one CU, so the step is bound by the per-frame update latency, not HBM'}}


def fte_iter_profile(frames):
    """The newest committed per-iteration profile of the FTE at `frames` frames
    (profiles/r*/fte_iter_<frames/1000>k.json, tools/fte_iter_json.py: rocprofv3 kernel times
    and the calibrated PMC HBM bytes of one LM iteration, per launch). None if not profiled."""
    import glob
    root = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(root, 'profiles', 'r*', f'fte_iter_{frames // 1000}k.json')))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    d['file'] = os.path.relpath(files[-1], root)
    return d


def fte_roofline(n_frames, iters, ms_per_solve, P, C, L, frames_profiled=None):
    """FP64 roofline of a whole FTE solve with the algorithmic flops of SURVEY.md §8(d) (per
    frame per GN step: 2 (2CL) P^2 for J^T J + ~80 kflop FK / Jacobian + 6 P^3 banded solve),
    plus, from the committed profile of one LM iteration at this size, the dominant kernel's
    share of the iteration and the HBM bytes per iteration against §8(d)'s algorithmic
    2,872 B per frame (C L (2 b + 1) observations + 4 P b state, b = 8)."""
    flop_frame = 2 * (2 * C * L) * P * P + 80e3 + 6 * P ** 3
    tfs = n_frames * iters * flop_frame / (ms_per_solve * 1e-3) / 1e12
    r = {'bound': 'fp64', 'achieved': tfs, 'peak': FP64_PEAK_TFS, 'unit': 'TFLOP/s', 'frac': tfs / FP64_PEAK_TFS,
         'flop_per_frame_step': flop_frame, 'note': 'whole solve (all kernels), algorithmic flops of SURVEY.md 8(d)'}
    prof = fte_iter_profile(n_frames)
    if prof:
        alg = n_frames * (C * L * 17 + 4 * P * 8)
        dom = prof['dominant']
        r.update({'traffic': prof['hbm_bytes_per_iter'], 'traffic_unit': 'B per LM iteration (PMC, calibrated)',
                  'algorithmic_bytes_per_iter': alg, 'traffic_vs_algorithmic': prof['hbm_bytes_per_iter'] / alg,
                  'kernel_us_per_iter': prof['kernel_us_per_iter'],
                  'dominant_kernel': {'kernel': dom['kernel'], 'share_of_iteration': dom['share'],
                                      'us_per_iter': dom['us'], 'hbm_bytes_per_iter': dom['hbm_bytes']},
                  'by_kernel_share': {k: round(v['share'], 4) for k, v in prof['by_kernel'].items()},
                  'profile_source': prof['file']})
    return r


def bench_fte_window(ctx, torch, stream, n_frames, world, rank, exchange='nccl', steps=3):
    """configs[3]: one FTE trajectory of `n_frames` frames; with W ranks its super-blocks
    are split into W frame windows (acinoset_amd.dist, one all-reduce per LM step over
    RCCL). Strong scaling: the total work is fixed. W = 1 runs acs_fte_solve. Inputs are
    resident in HBM on every rank before the timed solves (device pointers), and the solution
    is written to device tensors. A rank's handle is created once, before the timed region,
    and every timed solve restarts it (acs_fte_dist_reset): the timed region makes no
    allocation (the library's allocation counter is reported)."""
    import torch.distributed as tdist
    from acinoset_amd import _native
    from acinoset_amd import dist as adist
    seq, cams, meas, w, X0, table, qinv = _fte_problem(ctx, n_frames)
    import datetime
    # a bounded collective timeout: a broken exchange ends the leg instead of hanging the run
    group = tdist.new_group(backend=exchange, timeout=datetime.timedelta(minutes=3)) if world > 1 else None
    dv = torch.device('cuda', torch.cuda.current_device())
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dv, dt)  # noqa: E731
    dev = dict(ints=T(table.ints, torch.int32), reals=T(table.reals), cams=T(cams), meas=T(meas), w=T(w),
               qinv=T(qinv), X=T(X0), tau=torch.zeros(len(cams), dtype=torch.float64, device=dv))
    d_X = dev['X'].clone()
    d_tau = dev['tau'].clone()
    N, Cn = meas.shape[0], meas.shape[1]
    r = None
    if world > 1:
        r = adist.HipFteRank(ctx, table, cams, meas, w, seq.Ts, qinv, X0, rank=rank, world=world, dev=dev)
    allreduce = adist.torch_allreduce(group) if world > 1 else None

    def run():
        if world == 1:
            d_X.copy_(dev['X'])
            d_tau.zero_()
            rep = ctx.fte_solve_dev(dev['ints'].data_ptr(), len(table.ints), dev['reals'].data_ptr(), len(table.reals),
                                    dev['cams'].data_ptr(), Cn, dev['meas'].data_ptr(), dev['w'].data_ptr(), N, True,
                                    seq.Ts, dev['qinv'].data_ptr(), 1, d_X.data_ptr(), d_tau.data_ptr())
            return d_X, d_tau, rep
        r.reset(dev['X'], dev['tau'])
        adist.lm_loop([r], allreduce)
        return r.result(d_X, d_tau)
    try:
        X, tau, rep = run()                                         # warm-up (graphs captured) + result
        X, tau = X.cpu().numpy(), tau.cpu().numpy()
        pos = ctx.fk(table, X[2:])
        pos_rms = float(np.sqrt(np.mean(np.sum((pos - seq.pos3d[:, 0]) ** 2, -1))))
        if world > 1:
            tdist.barrier()
        torch.cuda.synchronize()
        a0 = _native.alloc_events()
        t0 = time.perf_counter()
        each = []
        for _ in range(steps):
            t1 = time.perf_counter()
            run()                                                   # returns after the solve
            each.append(time.perf_counter() - t1)
        torch.cuda.synchronize()
        if world > 1:
            tdist.barrier()
        dt = (time.perf_counter() - t0) / steps
        allocs = _native.alloc_events() - a0
    finally:
        if r is not None:
            r.close()
    if world > 1:
        t = torch.tensor([dt, float(allocs)], dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt, allocs = float(t[0].item()), int(t[1].item())
    L = table.L
    out = {'workload': f'fte C={Cn} frames={n_frames} L={L} P={table.P} sd=const intermode=vel (configs[3])',
           'ranks': world, 'scaling': 'strong', 'frames_per_s': n_frames / dt, 'ms_per_solve': dt * 1e3,
           'ms_per_solve_each_rank0': [round(e * 1e3, 3) for e in each],
           'status': rep['status_name'], 'iters': rep['iters'], 'cost_after': rep['cost_after'],
           'pos_rms_vs_truth_m': pos_rms, 'tau_err_max_s': float(np.abs(tau - seq.tau).max()),
           'alloc_events_in_timed_region': allocs,
           'exchange': 'none' if world == 1 else (f'torch.distributed {exchange}: one all-reduce per LM step '
                                                   '(chain-end reduced system + trial cost, one payload) + the '
                                                   'solution rows once')}
    out['roofline'] = fte_roofline(n_frames, rep['iters'], dt * 1e3, table.P, Cn, L)
    if world > 1:
        out['roofline'].pop('traffic', None)      # the committed profile is of the single-GPU iteration
        out['roofline']['note'] += '; per-iteration profile fields are of the single-GPU solve'
    return out


def fte_cpu_baseline(wl):
    """Oracle FTE (oracle/fte.py: numpy float64, banded Cholesky + tau Schur complement per
    LM step, 1 core: the LM is a sequential chain of banded factorisations) on the whole
    configs[2] problem from the same start, solved once to the same LM stop. Returns
    (baseline dict, (X, tau, info)) - the solution is the oracle side of the bench's
    reprojection parity."""
    from oracle import fte as ofte
    sc = wl.scene
    model, _ = host_cpu()
    prob = ofte.Problem('default_nolure', wl.meas, wl.w, sc.K, sc.D, sc.R, sc.t, wl.Ts, sd=True, intermode='vel')
    t0 = time.perf_counter()
    X, tau, info = ofte.solve(prob, wl.X0)
    dt = time.perf_counter() - t0
    N = wl.meas.shape[0]
    return ({'value': N / dt, 'unit': 'frames/s', 'cores': 1, 'cpu_model': model, 'kind': 'port',
             'sample': f'one full solve of the same {N}-frame problem ({info["iters"]} LM iterations, status '
                       f'{info["status"]}; oracle/fte.py, numpy float64 + LAPACK banded Cholesky), {dt:.1f} s'},
            (X, tau, info))


def bench_fte(ctx, torch, stream, n_frames=1000, steps=5, cpu=True):
    """configs[2]: 6-cam x 1000-frame FTE (20 keypoints, P = 26, shutter delay 'const',
    interpolation 'vel' = the all_optimizations defaults, src/all_optimizations.py:127-136),
    from the reference initialisation (pairwise triangulation on the GPU + nose line fit,
    acinoset_amd.workloads). With `cpu`, the oracle solves the same problem once (timed:
    cpu_baseline) and the reprojection RMS of both solutions is reported."""
    from acinoset_amd import workloads
    wl = workloads.fte_workload(ctx, n_frames)
    table, C = wl.table, wl.cams.shape[0]
    N, _, L, _ = wl.meas.shape
    dev = torch.device('cuda', torch.cuda.current_device())
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    d_ints, d_reals, d_cams, d_meas, d_w, d_q = (T(table.ints, torch.int32), T(table.reals), T(wl.cams), T(wl.meas),
                                                 T(wl.w), T(wl.qinv))
    d_X0, d_X, d_tau = T(wl.X0), T(wl.X0), torch.zeros(C, dtype=torch.float64, device=dev)
    opts = ctx.fte_default_opts()

    def run():
        d_X.copy_(d_X0)
        d_tau.zero_()
        return ctx.fte_solve_dev(d_ints.data_ptr(), len(table.ints), d_reals.data_ptr(), len(table.reals),
                                 d_cams.data_ptr(), C, d_meas.data_ptr(), d_w.data_ptr(), N, True, wl.Ts,
                                 d_q.data_ptr(), 1, d_X.data_ptr(), d_tau.data_ptr(), opts)
    rep = run()                                                    # warm-up + correctness
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        rep = run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    X = d_X.cpu().numpy()
    tau = d_tau.cpu().numpy()
    pos = ctx.fk(table, X[2:])
    pos_rms = float(np.sqrt(np.mean(np.sum((pos - wl.seq.pos3d[:, 0]) ** 2, -1))))
    rms = workloads.fte_reproj_rms(ctx, wl, X, tau)
    out = {'workload': f'fte C={C} frames={N} L={L} P={table.P} sd=const intermode=vel (configs[2])',
           'frames_per_s': N / dt, 'ms_per_solve': dt * 1e3, 'status': rep['status_name'], 'iters': rep['iters'],
           'accepted': rep['n_accepted'], 'cost_before': rep['cost_before'], 'cost_after': rep['cost_after'],
           'reproj_rms_px': rms, 'pos_rms_vs_truth_m': pos_rms,
           'tau_err_max_s': float(np.abs(tau - wl.seq.tau).max()),
           'roofline': fte_roofline(N, rep['iters'], dt * 1e3, table.P, C, L)}
    if cpu:
        out['cpu_baseline'], (Xo, to, info) = fte_cpu_baseline(wl)
        ro = workloads.fte_reproj_rms(ctx, wl, Xo, to)
        po = ctx.fk(table, np.ascontiguousarray(Xo[2:]))
        out['reproj_rms_oracle_px'] = ro
        out['reproj_rms_vs_oracle_px'] = rms - ro
        out['kp_rms_vs_oracle_m'] = float(np.sqrt(np.mean(np.sum((pos - po) ** 2, -1))))
        out['oracle'] = {'status': info['status'], 'iters': info['iters'], 'cost_after': float(info['cost_after']),
                         'tau_max_diff_s': float(np.abs(tau - to).max())}
    return out


if __name__ == '__main__':
    main()
