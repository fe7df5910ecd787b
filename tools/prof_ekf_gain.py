"""Phase times of k_ekf_gain_t (the 87-state RTS gains) in the bench's default-model EKF call
(64 sequences x 500 frames, 12 cameras), from a library built with -DEKF_PROFILE
(tools/build_prof.sh ekf): python tools/prof_ekf_gain.py [seqs] [frames]. Per workgroup: load,
Gauss-Jordan and product time; the kernel's span and the workgroups in flight it implies."""
import ctypes as C
import os
import sys

os.environ['ACINOSET_HIP_LIB'] = os.environ.get('ACS_PROF_LIB') or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), '..', 'acinoset_amd', 'csrc', 'build', 'libprof.so')
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

seqs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 500
ctx = _native.Context(0)
fn = ctx.lib.acs_ekf_gain_prof
fn.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
bench.bench_ekf(ctx, torch, seqs, frames, 12, 1, 0, mode='default', steps=1)   # warm-up
fn(buf, 1)
bench.bench_ekf(ctx, torch, seqs, frames, 12, 1, 0, mode='default', steps=1)
torch.cuda.synchronize()
fn(buf, 0)
v = np.array(buf[:], np.float64)
n = max(v[3], 1)
print(f'workgroups {int(v[3])} (over the calls of one bench_ekf: warm-up, timed, check)')
for k, nm in enumerate(('load P_pred / P_est F^T', 'Gauss-Jordan inverse', 'product + store')):
    print(f'{nm:26s} {v[k] / n * 1e-2:8.2f} us per workgroup')
# the last launch's workgroups: how many are in flight over time
tr = (C.c_ulonglong * (2 * 32768))()
ctx.lib.acs_ekf_gain_trace.argtypes = [C.c_void_p]
ctx.lib.acs_ekf_gain_trace(tr)
t = np.array(tr[:], np.int64).reshape(-1, 2)
t = t[(t[:, 0] > 0) & (t[:, 1] > t[:, 0])]
t0 = t[:, 0].min()
ent, ex = (t[:, 0] - t0) * 1e-2, (t[:, 1] - t0) * 1e-2
span = ex.max()
print(f'last launch: {len(t)} workgroups traced, span {span:.0f} us, mean life {np.mean(ex - ent):.1f} us, '
      f'mean in flight {np.sum(ex - ent) / span:.0f}')
nb = int(span) + 1
alive = np.zeros(nb)
for a, b in zip(ent.astype(int), ex.astype(int)):
    alive[a:b + 1] += 1
print('in flight per 100 us:', ' '.join(str(int(x)) for x in alive[::100]))
