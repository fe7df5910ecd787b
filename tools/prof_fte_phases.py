"""Per-phase wall-clock split of k_cr_level (block 0 of each launch), from a library built
with -DFTE_PROFILE:
  B=acinoset_amd/csrc/build; hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -DFTE_PROFILE \
     -c acinoset_amd/csrc/fte.hip -o $B/fte_prof.o && hipcc --offload-arch=gfx950 -shared -fPIC \
     $B/{ctx,ekf,fk,sba,sba_ext,tri,pipeline}.o $B/fte_prof.o -o $B/libprof.so
then python tools/prof_fte_phases.py [frames]."""
import ctypes as C
import os
import sys

os.environ['ACINOSET_HIP_LIB'] = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'acinoset_amd',
                                              'csrc', 'build', 'libprof.so')
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

ctx = _native.Context(0)
seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
buf = (C.c_ulonglong * 32)()
ctx.lib.acs_fte_prof_read.argtypes = [C.c_void_p]
X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0)
ctx.lib.acs_fte_prof_read(buf)
v = np.array(buf[:], np.float64) * 10e-3   # 100 MHz ticks -> us
n = rep['iters'] * 9                        # elimination launches (9 levels at 1000 frames)
names = {0: 'load (+pending, LDS copies)', 1: 'Gauss-Jordan', 3: 'W store + left terms (wave NB)',
         4: 'right terms (wave NB)', 11: 'W store + left terms (wave 15)', 12: 'right terms (wave 15)',
         13: 'Tau (wave 15)'}
print(f"iters {rep['iters']}; us per elimination launch (block 0):")
for k, nm in names.items():
    print(f'{nm:32s} {v[k] / n:8.2f}')
