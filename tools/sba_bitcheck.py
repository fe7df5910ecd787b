"""Bitwise A/B of two builds of the SBA kernel: run the headline problem and the configs[4]-shape one
with the library named by
ACINOSET_HIP_LIB; save the solutions and per-point status for a bitwise comparison."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np
import torch
from acinoset_amd import _native, workloads, synth
tag = sys.argv[1]
ctx = _native.Context(0)
dev = torch.device('cuda', 0)
out = {}
wl = workloads.sba_reference_workload()
probs = [('cfg1', wl.cams, wl.uv, wl.mask, wl.pts0)]
scene = synth.ring_scene(12)
seq = synth.make_sequence(20000, scene, mode='default_nolure', seed=4242)
uv, mask, pts0, truth, _ = synth.dense_sba_problem(seq)
probs.append(('cfg4', _native.pack_cameras(scene.K, scene.D, scene.R, scene.t), uv, mask, pts0))
for name, cams, uv, mask, pts0 in probs:
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_cams, d_uv, d_mask, d_pts0 = T(cams), T(uv), T(mask), T(pts0)
    d_pts = d_pts0.clone()
    n_pts, C = mask.shape
    opts = _native.Context.sba_opts()
    rep = ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts, d_pts.data_ptr(),
                                   opts, report=True, pts_in_p=d_pts0.data_ptr())
    out[name] = d_pts.cpu().numpy()
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            ctx.sba_points_dense_dev(d_cams.data_ptr(), C, d_uv.data_ptr(), d_mask.data_ptr(), n_pts, d_pts.data_ptr(),
                                     opts, pts_in_p=d_pts0.data_ptr())
        e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e) / 50)
    print(tag, name, 'ms per solve', ['%.4f' % t for t in ts], 'iters', rep['iters_max'] if 'iters_max' in rep else rep, flush=True)
os.makedirs('gpurun_out', exist_ok=True)
np.savez(f'gpurun_out/sba_bits_{tag}.npz', **out)
if tag == 'new' and os.path.exists('gpurun_out/sba_bits_head.npz'):
    h = np.load('gpurun_out/sba_bits_head.npz')
    for k in out:
        print(k, 'bit-identical' if np.array_equal(h[k].view(np.uint64), out[k].view(np.uint64)) else
              f'DIFFER max {np.abs(h[k] - out[k]).max():.3e}')
