"""One bench EKF leg on its own (bench.bench_ekf): python tools/time_ekf_leg.py [mode] [jacobian]
[seqs] [frames]; run under rocprofv3 --kernel-trace for the per-kernel times."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else 'default'
jac = sys.argv[2] if len(sys.argv) > 2 else 'fd'
seqs = int(sys.argv[3]) if len(sys.argv) > 3 else 64
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 500
ctx = _native.Context(0)
stream = torch.cuda.Stream(device=0)   # as bench.main: the context's stream is torch's current one
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
r = bench.bench_ekf(ctx, torch, seqs, frames, 12, 1, 0, mode=mode, steps=3, jacobian=jac)
print(json.dumps(r))
