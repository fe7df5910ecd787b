import sys, ctypes as C, numpy as np, importlib, torch
sys.path.insert(0, '.')
from acinoset_amd import _native, synth, kinematics as pkin
cekf = importlib.import_module('acinoset_amd.core.ekf')
ctx = _native.Context(0)
buf = torch.zeros(8, dtype=torch.int64, device='cuda')
ctx.lib.acs_ekf_prof.argtypes = [C.c_void_p]
ctx.lib.acs_ekf_prof(C.c_void_p(buf.data_ptr()))
mode, N = 'default', 200
scene = synth.load_scene_file(); seq = synth.make_sequence(N, scene, mode=mode, seed=5)
table = pkin.build_table(mode); cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t); P = table.P
s0 = np.zeros(3 * P); s0[:3] = seq.pos3d[0, 0, 0]
ctx.ekf_run(table, cams, seq.uv, seq.likelihood, 90.0, 0.5, 2704.0, cekf.measurement_std(6), cekf.process_covariance(P, 1/90.), cekf.initial_covariance(mode), s0)
v = buf.cpu().numpy() / N
names = ["predict+PFPt", "FK/proj", "H build", "A,G,b,outl", "aug", "GJ", "update", "store+FK-only"]
for nm, x in zip(names, v): print(f'{nm:12s} {x:10.0f} cycles/frame  ({x/2.4e3:.1f} us @2.4GHz)')
