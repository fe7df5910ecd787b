"""Timeline of one deep k_cr_level launch (block 0, levels with ne * nsplit <= 12; with
-DFTE_PROF_WIDE=n the levels with >= n elimination workgroups instead), from a library built
with -DFTE_PROFILE (see tools/prof_fte_phases.py for the build line):
python tools/prof_cr_timeline.py [frames]. Prints the mean time since the kernel start of
each event."""
import ctypes as C
import os
import sys

os.environ['ACINOSET_HIP_LIB'] = os.environ.get('ACS_PROF_LIB') or os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'acinoset_amd',
                                              'csrc', 'build', 'libprof.so')
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

ctx = _native.Context(0)
seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
buf = (C.c_ulonglong * 64)()
ctx.lib.acs_fte_prof_read.argtypes = [C.c_void_p]
X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0)
ctx.lib.acs_fte_prof_read(buf)
n = max(buf[63], 1)
v = np.array(buf[:], np.float64) * 10e-3 / n   # 100 MHz ticks -> us, per launch
names = {32: 'wave 0 loads done', 33: 'col wave loads done', 34: 'pivot 0 inv+row', 35: 'pivot 1', 36: 'pivot 2',
         37: 'pivot 3', 38: 'pivot 4', 39: 'pivot 5', 40: 'col wave GJ done', 41: 'left term done',
         42: 'right term done', 43: 'Tau done', 29: 'wave 15 GJ done', 30: 'wave 15 Schur done',
         31: 'row wave 0 GJ done'}
# next pivot wave: after the barrier (44 + k) and after its inverse (50 + k)
for k in range(4):
    names[44 + k] = f'pivot {k + 1} start (after barrier)'
    names[50 + k] = f'pivot {k + 1} inverse done'
print(f'profiled launches {buf[63]}; mean us since kernel start:')
for k, nm in sorted(names.items(), key=lambda kv: v[kv[0]]):
    print(f'{nm:24s} {v[k]:8.2f}')
