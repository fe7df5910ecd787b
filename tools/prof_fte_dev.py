"""The bench's configs[2] FTE leg (resident inputs, acs_fte_solve_dev) repeated, for
rocprofv3 --kernel-trace: where a solve's wall time goes between and around the LM
iterations. Prints each solve's host time; tools/fte_solve_timeline.py reads the trace.
python tools/prof_fte_dev.py [frames] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acinoset_amd import _native, workloads  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = _native.Context(0)
wl = workloads.fte_workload(ctx, N)
table, C = wl.table, wl.cams.shape[0]
dev = torch.device('cuda', 0)
T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
d_ints, d_reals, d_cams, d_meas, d_w, d_q = (T(table.ints, torch.int32), T(table.reals), T(wl.cams), T(wl.meas),
                                             T(wl.w), T(wl.qinv))
d_X0, d_X, d_tau = T(wl.X0), T(wl.X0), torch.zeros(C, dtype=torch.float64, device=dev)
opts = ctx.fte_default_opts()
for r in range(reps + 1):
    d_X.copy_(d_X0)
    d_tau.zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    rep = ctx.fte_solve_dev(d_ints.data_ptr(), len(table.ints), d_reals.data_ptr(), len(table.reals),
                            d_cams.data_ptr(), C, d_meas.data_ptr(), d_w.data_ptr(), wl.meas.shape[0], True, wl.Ts,
                            d_q.data_ptr(), 1, d_X.data_ptr(), d_tau.data_ptr(), opts)
    torch.cuda.synchronize()
    print(f'solve {r}: {1e3 * (time.perf_counter() - t):.3f} ms host, {rep["iters"]} iterations', flush=True)
