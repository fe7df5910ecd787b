"""configs[2] oracle LM history (cost, lambda, step) on the GPU-built workload, and the
iteration count / final cost / reprojection under other damping schedules (experiment)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from acinoset_amd import _native, workloads
from oracle import fte as ofte

ctx = _native.Context(0)
wl = workloads.fte_workload(ctx, int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
sc = wl.scene
prob = ofte.Problem('default_nolure', wl.meas, wl.w, sc.K, sc.D, sc.R, sc.t, wl.Ts, sd=True, intermode='vel')
for lam0 in (1e-3, 1e-5):
    t0 = time.perf_counter()
    X, tau, info = ofte.solve(prob, wl.X0, lam0=lam0, verbose=True)
    print(f'lam0 {lam0}: {info["status"]} iters {info["iters"]} acc {info["n_accepted"]} F {info["cost_after"]:.12e} '
          f'reproj {workloads.fte_reproj_rms(ctx, wl, X, tau):.9f} px, {time.perf_counter() - t0:.1f} s', flush=True)
