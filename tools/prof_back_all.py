"""Per-workgroup timeline of the last k_cr_back_all launch of one FTE solve, from a library
built with -DFTE_PROFILE (tools/build_prof.sh fte): python tools/prof_back_all.py [frames].
Per level: workgroup count, first entry / last end since the launch's first entry, mean
wait for the inputs (entry -> every granule carries the stamp) and mean work after them.
Levels 100 / 101 are the tau partial chunks and the top block."""
import ctypes as C
import os
import sys

os.environ['ACINOSET_HIP_LIB'] = os.environ.get('ACS_PROF_LIB') or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), '..', 'acinoset_amd', 'csrc', 'build', 'libprof.so')
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from acinoset_amd import _native  # noqa: E402

NT = 8192
ctx = _native.Context(0)
seq, cams, meas, w, X0, table, qinv = bench._fte_problem(ctx, int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
X, tau, rep = ctx.fte_solve(table, cams, meas, w, seq.Ts, qinv, X0)
buf = (C.c_ulonglong * (4 * NT))()
ctx.lib.acs_fte_back_trace_read.argtypes = [C.c_void_p]
ctx.lib.acs_fte_back_trace_read(buf)
t = np.array(buf[:], np.int64).reshape(NT, 4)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
ent, rdy, end, lv = (t[:, 0] - t0) * 1e-2, (t[:, 1] - t0) * 1e-2, (t[:, 2] - t0) * 1e-2, t[:, 3]
rdy = np.where(t[:, 1] > 0, rdy, ent)
print(f'{len(t)} workgroups, span {end.max():.2f} us (100 MHz clock)')
print(f"{'level':>6} {'n':>5} {'first in':>9} {'last in':>9} {'last end':>9} {'wait':>7} {'work':>7} {'life':>7}")
for L in sorted(set(lv.tolist()), key=lambda x: (x < 100, -x)):
    m = lv == L
    print(f'{L:6d} {m.sum():5d} {ent[m].min():9.2f} {ent[m].max():9.2f} {end[m].max():9.2f} '
          f'{(rdy[m] - ent[m]).mean():7.2f} {(end[m] - rdy[m]).mean():7.2f} {(end[m] - ent[m]).mean():7.2f}')
# residency: workgroups alive per 1 us bin
nb = int(np.ceil(end.max())) + 1
alive = np.zeros(nb)
for a, b in zip(ent, end):
    alive[int(a):int(b) + 1] += 1
print('alive per us (every 5th bin):', ' '.join(f'{int(x)}' for x in alive[::5]))
