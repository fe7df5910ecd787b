"""Per-phase cycle counts of k_ekf_filter from a library built with -DEKF_PROFILE (the same
libprof.so as tools/prof_fte_phases.py, with ekf.hip compiled with -DEKF_PROFILE):
python tools/prof_ekf_phases.py [mode] [n_cams] [frames] [fd|analytic]   (default: default 6 200 fd;
'fd' = the reference numerics with the forward-difference H, 'analytic' = the analytic H in float64).
Build: tools/build_prof.sh ekf (rebuild after every ekf.hip change; ACS_PROF_LIB=<path> picks another
profiling build)."""
import ctypes as C
import importlib
import os
import sys

os.environ['ACINOSET_HIP_LIB'] = os.environ.get('ACS_PROF_LIB') or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), '..', 'acinoset_amd', 'csrc', 'build', 'libprof.so')
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from acinoset_amd import _native, synth, kinematics as pkin  # noqa: E402

cekf = importlib.import_module('acinoset_amd.core.ekf')
mode = sys.argv[1] if len(sys.argv) > 1 else 'default'
n_cams = int(sys.argv[2]) if len(sys.argv) > 2 else 6
N = int(sys.argv[3]) if len(sys.argv) > 3 else 200
jac = sys.argv[4] if len(sys.argv) > 4 else 'fd'
ctx = _native.Context(0)
buf = torch.zeros(9, dtype=torch.int64, device='cuda')
ctx.lib.acs_ekf_prof.argtypes = [C.c_void_p]
ctx.lib.acs_ekf_prof(C.c_void_p(buf.data_ptr()))
scene = synth.load_scene_file() if n_cams == 6 else synth.ring_scene(n_cams)
seq = synth.make_sequence(N, scene, mode=mode, seed=5)     # as bench.py's EKF leg
table = pkin.build_table(mode)
cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t)
P = table.P
covs = cekf.ring_cal_covs(n_cams)
s0 = np.zeros((1, 3 * P))
s0[0, :P] = seq.x[0]
s0[0, P:2 * P] = (seq.x[1] - seq.x[0]) / seq.Ts
ctx.ekf_run(table, cams, seq.uv[None], seq.likelihood[None],
            90.0, 0.5, float(scene.res[0]), cekf.measurement_std(n_cams, covs), cekf.process_covariance(P, 1 / 90.),
            cekf.initial_covariance(mode), s0, ref_numerics=jac == 'fd', jacobian=jac)
v9 = buf.cpu().numpy() / N
v, sub = v9[:8], v9[8]
names = ["predict+PFPt", "FK/proj", "H build", "A,G,b,outl", "aug", "GJ", "update", "store+FK-only"]
print(f'{mode}, {n_cams} cams, {N} frames, one sequence, H: {jac}')
for nm, x in zip(names, v):
    print(f'{nm:14s} {x:10.0f} cycles/frame  ({x / 2.4e3:.1f} us @2.4GHz)')
print(f'{"total":14s} {v.sum():10.0f} cycles/frame  ({v.sum() / 2.4e3:.1f} us @2.4GHz)')
if sub:  # k_ekf_filter_w1, one-joint skeletons: the trig / translation tables inside FK/proj
    print(f'{"  FK/proj: trig":14s} {sub:10.0f} cycles/frame  ({sub / 2.4e3:.1f} us @2.4GHz)')
