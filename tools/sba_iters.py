"""Kernel time of the configs[1] SBA solve (acs_sba_points_dense_io, HIP events on the
kernel stream) against the LM iteration cap: fixed cost and per-iteration slope.
    python tools/sba_iters.py"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np
import torch
from acinoset_amd import _native, synth
ctx = _native.Context(0)
torch.cuda.set_device(0)
stream = torch.cuda.Stream(device=0)
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
scene = synth.load_scene_file()
seq = synth.make_sequence(100, scene, mode='default_nolure', seed=0)
uv, mask, pts0, truth, _ = synth.dense_sba_problem(seq)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
n_pts, C = mask.shape
dev = torch.device('cuda', 0)
d_cams, d_uv, d_mask, d_pts0 = (torch.from_numpy(a).to(dev) for a in (cams, uv, mask, pts0))
d_pts = d_pts0.clone()
fn = ctx.lib.acs_sba_points_dense_io
for mi in [0, 1, 2, 3, 4, 5, 6, 7, 8, 100]:
    opts = _native.Context.sba_opts(max_iters=mi)
    call = (ctx.h, ctypes.c_void_p(d_cams.data_ptr()), C, ctypes.c_void_p(d_uv.data_ptr()),
            ctypes.c_void_p(d_mask.data_ptr()), n_pts, ctypes.c_void_p(d_pts0.data_ptr()),
            ctypes.c_void_p(d_pts.data_ptr()), ctypes.byref(opts), None, _native.ACS_DEVICE_PTRS)
    for _ in range(20):
        rc = fn(*call)
        assert rc == 0, (rc, ctx.lib.acs_last_error(ctx.h))
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(200):
        fn(*call)
    b.record(stream)
    torch.cuda.synchronize()
    print(f'max_iters {mi:3d}: {a.elapsed_time(b) / 200 * 1e3:7.2f} us per solve', flush=True)
