"""FTE solve only (configs[2] by default), for rocprofv3 --kernel-trace per-dispatch timing:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ftetrace -o run -- python3 tools/prof_fte.py
and tools/fte_trace_summary.py on the CSV."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--frames', type=int, default=1000)
ap.add_argument('--reps', type=int, default=3)
ap.add_argument('--sd-mode', default='const')
a = ap.parse_args()
ctx = _native.Context(0)
seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, a.frames)
for r in range(a.reps):
    t = time.perf_counter()
    X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0, sd_mode=a.sd_mode)
    print(f"rep {r}: {1e3 * (time.perf_counter() - t):.2f} ms, iters {rep['iters']}, {rep['status_name']}",
          flush=True)
