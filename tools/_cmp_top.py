"""Old vs new CR top: max |X - oracle| for the variable-delay LM-step test cases."""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np
from acinoset_amd import _native, kinematics as pkin
from oracle import fte as ofte
import test_gpu_fte as T
ctx = _native.Context(0)
for N, iters in [(31, 1), (31, 3), (31, 5), (31, 8), (64, 5)]:
    for sd in ('variable', 'const'):
        seq, prob, cams = T._problem(N, sd_mode=sd)
        X0 = ofte.initial_state(prob, np.arange(N), seq.pos3d[:, 0, 0])
        table = pkin.build_table(prob.mode)
        X, tau, rep = ctx.fte_solve(table, cams, prob.meas, prob.w, prob.Ts, prob.qinv, X0,
                                    opts=ctx.fte_default_opts(max_iters=iters), sd_mode=sd)
        Xo, to, info = ofte.solve(prob, X0, max_iters=iters)
        print(os.environ.get('ACINOSET_HIP_LIB', 'new')[-12:], sd, N, iters, 'max|X-Xo| %.3e' % np.abs(X - Xo).max(), flush=True)
