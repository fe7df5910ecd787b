import sys, time, importlib, numpy as np
sys.path.insert(0, '.')
from acinoset_amd import _native, synth, kinematics as pkin
cekf = importlib.import_module('acinoset_amd.core.ekf')
ctx = _native.Context(0)
for mode in ['head', 'default']:
    scene = synth.load_scene_file(); seq = synth.make_sequence(3, scene, mode=mode, seed=5)
    table = pkin.build_table(mode); cams = _native.pack_cameras(scene.K, scene.D, scene.R, scene.t); P = table.P
    s0 = np.zeros(3 * P); s0[:3] = seq.pos3d[0, 0, 0]
    print(mode, 'start', flush=True)
    t = time.time()
    out = ctx.ekf_run(table, cams, seq.uv, seq.likelihood, 90.0, 0.5, 2704.0, cekf.measurement_std(6), cekf.process_covariance(P, 1/90.), cekf.initial_covariance(mode), s0)
    print(mode, 'done', time.time() - t, out['x_est'][-1, :3], flush=True)
