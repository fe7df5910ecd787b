"""Phase timeline of k_fte_linearize (block 0) from a -DFTE_PROFILE library (see
tools/prof_fte_phases.py for the build line): python tools/prof_lin_phases.py [frames]."""
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
buf = (C.c_ulonglong * 64)()
ctx.lib.acs_fte_prof_read.argtypes = [C.c_void_p]
X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0)
ctx.lib.acs_fte_prof_read(buf)
n = max(buf[60], 1)
v = np.array(buf[:], np.float64) * 10e-3 / n
print(f'linearize launches {buf[60]}; block 0, mean us since kernel start:')
fk = [(24, 'sincos'), (25, 'barrier 1'), (26, 'joint rotations G'), (27, 'joint frames M (chains)'),
      (28, 'node positions')]
print('fk_frame (thread 0, block 0), mean us since fk_frame start:')
for k, nm in fk:
    print(f'  {nm:32s} {v[k]:8.2f}')
print('phase (b), summed over the marker chunks:')
for k, nm in [(14, 'operand rows (fk_dpos, Z D + Q)'), (15, 'gradient + MFMA + barrier')]:
    print(f'  {nm:32s} {v[k]:8.2f}')
for k, nm in [(61, 'skeleton table staged'), (62, 'cams / LDS init (FK start)'), (56, 'FK done'), (57, 'observations + aggregation done'), (58, 'MFMA H done'), (59, 'store done')]:
    print(f'{nm:34s} {v[k]:8.2f}')
