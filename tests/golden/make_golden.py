"""Generate the golden fixtures under tests/golden/ by running the REFERENCE code.

Runs in the build container only (the reference is not on the GPU box). The
reference's own `src/lib/sba.py`, `src/lib/utils.py`, `src/lib/calib.py`,
`src/lib/metric.py` and `src/lib/misc.py` are imported from /root/reference/src;
the four OpenCV calls go through `_cv2shim` (cv2 is not installed).

Inputs come from the build's seeded synthetic generator (`acinoset_amd.synth`).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = os.environ.get('ACINOSET_REF_SRC', '/root/reference/src')
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import _cv2shim  # noqa: E402

_cv2shim.install()
sys.path.insert(0, REF_SRC)

from lib import misc as ref_misc      # noqa: E402  (reference)
from lib import sba as ref_sba        # noqa: E402
from lib import utils as ref_utils    # noqa: E402
from lib import calib as ref_calib    # noqa: E402
from lib import metric as ref_metric  # noqa: E402

from acinoset_amd import synth        # noqa: E402


def _df_arrays(df, markers):
    mi = {m: i for i, m in enumerate(markers)}
    return dict(df_frame=df['frame'].to_numpy(np.int64), df_camera=df['camera'].to_numpy(np.int64),
                df_marker=np.array([mi[m] for m in df['marker']], np.int64),
                df_x=df['x'].to_numpy(np.float64), df_y=df['y'].to_numpy(np.float64),
                df_likelihood=df['likelihood'].to_numpy(np.float64))


def sba_fixture(name, n_frames, cams, thresh=0.5, seed=0):
    scene = synth.load_scene_file().subset(cams)
    seq = synth.make_sequence(n_frames, scene, mode='default_nolure', seed=seed)
    df = seq.to_df()
    df = df.query(f'likelihood > {thresh}')                    # src/core/sba.py:41
    df = df[df['frame'].between(0, n_frames - 1)].reset_index(drop=True)
    scene_path = os.path.join('/tmp', f'golden_{name}_scene.json')
    scene.to_json(scene_path)

    captured = {}
    orig = ref_sba.bundle_adjust_points_only

    def spy(points_2d, points_3d, point_3d_indices, camera_indices, *a, **k):
        captured.update(points_2d=np.array(points_2d, np.float64), points_3d=np.array(points_3d, np.float64),
                        point_indices=np.array(point_3d_indices, np.int64),
                        camera_indices=np.array(camera_indices, np.int64))
        return orig(points_2d, points_3d, point_3d_indices, camera_indices, *a, **k)

    ref_sba.bundle_adjust_points_only = spy
    t0 = time.time()
    try:
        pts_df, res = ref_sba._sba_points(scene_path, df, ref_calib.triangulate_points_fisheye,
                                          ref_calib.project_points_fisheye)
    finally:
        ref_sba.bundle_adjust_points_only = orig
    dt = time.time() - t0
    markers = seq.markers
    mi = {m: i for i, m in enumerate(markers)}
    out = dict(K=scene.K, D=scene.D, R=scene.R, t=scene.t, res=np.array(scene.res),
               thresh=thresh, n_frames=n_frames, ref_seconds=dt, **_df_arrays(df, markers),
               pts_frame=pts_df['frame'].to_numpy(np.int64),
               pts_marker=np.array([mi[m] for m in pts_df['marker']], np.int64),
               pts_out=pts_df[['x', 'y', 'z']].to_numpy(np.float64),
               resid_before=np.asarray(res['before'], np.float64),
               resid_after=np.asarray(res['after'], np.float64), **captured)
    # parity metric: src/lib/metric.py:36 on the SBA output (cast to float)
    camera_params = (scene.K, scene.D, scene.R, scene.t, scene.res, len(cams))
    err = ref_metric.residual_error(df, pts_df, markers, camera_params)
    allres = []
    for c in range(len(cams)):
        e = err[str(c)]
        if e is not None and len(e):
            allres.append(e['pixel_residual'].astype(float).to_numpy())
    out['metric_pixel_residual'] = np.concatenate(allres) if allres else np.zeros(0)
    np.savez_compressed(os.path.join(HERE, f'{name}.npz'), **out)
    print(f'{name}: {len(out["points_2d"])} obs, {len(out["points_3d"])} pts, ref solve {dt:.2f}s')


def triangulation_fixture():
    scene = synth.load_scene_file()
    seq = synth.make_sequence(8, scene, mode='default_nolure', seed=11)
    df = seq.to_df().query('likelihood > 0.5').reset_index(drop=True)
    pts = ref_utils.get_pairwise_3d_points_from_df(df, scene.K, scene.D.reshape((-1, 4)), scene.R, scene.t,
                                                   ref_calib.triangulate_points_fisheye, verbose=False)
    mi = {m: i for i, m in enumerate(seq.markers)}
    # single-pair triangulation and undistortion samples
    a = df[df['camera'] == 0]
    b = df[df['camera'] == 1]
    j = a.merge(b, on=['frame', 'marker'], suffixes=('_a', '_b'))
    pa = j[['x_a', 'y_a']].to_numpy(np.float64)
    pb = j[['x_b', 'y_b']].to_numpy(np.float64)
    tri01 = ref_calib.triangulate_points_fisheye(pa, pb, scene.K[0], scene.D[0], scene.R[0], scene.t[0],
                                                 scene.K[1], scene.D[1], scene.R[1], scene.t[1])
    np.savez_compressed(os.path.join(HERE, 'triangulation.npz'), K=scene.K, D=scene.D, R=scene.R, t=scene.t,
                        **_df_arrays(df, seq.markers),
                        out_frame=pts['frame'].to_numpy(np.int64),
                        out_marker=np.array([mi[m] for m in pts['marker']], np.int64),
                        out_xyz=pts[['x', 'y', 'z']].to_numpy(np.float64),
                        pair_a=pa, pair_b=pb, pair_xyz=np.asarray(tri01, np.float64))
    print('triangulation:', len(pts), 'points')


def fk_fixture():
    rng = np.random.default_rng(123)
    out = {}
    for mode in ('default', 'head', 'upper_body', 'head_stabilize'):
        P = len(ref_misc.get_pose_params(mode))
        n = 16
        x = rng.normal(0, 0.4, (n, P))
        x[:, :3] += [1.9, 6.4, 0.6]
        dx = rng.normal(0, 2.0, (n, P))
        ddx = rng.normal(0, 20.0, (n, P))
        tau = rng.uniform(-0.01, 0.01, n)
        for inter in ('pos', 'vel', 'acc'):
            for dirs in (False, True):
                if mode != 'default' and dirs is False and inter != 'pos':
                    pass
                res = np.array([ref_misc.get_3d_marker_coords({'x': x[i], 'dx': dx[i], 'ddx': ddx[i]}, tau[i],
                                                              directions=dirs, mode=mode, intermode=inter)
                                for i in range(n)], np.float64)
                out[f'{mode}_{inter}_{int(dirs)}'] = res
        out[f'{mode}_x'] = x
        out[f'{mode}_dx'] = dx
        out[f'{mode}_ddx'] = ddx
        out[f'{mode}_tau'] = tau
    np.savez_compressed(os.path.join(HERE, 'fk.npz'), **out)
    print('fk: done')


def loss_fixture():
    e = np.concatenate([np.linspace(-30, 30, 1201), np.array([0.0, 1e-6, -1e-6, 0.0589, 2.9999, 3.0, 10.0, 20.0, 25.0])])
    v = np.array([ref_misc.redescending_loss(x, 3, 10, 20) for x in e], np.float64)
    np.savez_compressed(os.path.join(HERE, 'loss.npz'), err=e, loss=v, a=3.0, b=10.0, c=20.0)
    print('loss: done')


def extrinsics_fixture(n_frames=4):
    scene = synth.load_scene_file()
    seq = synth.make_sequence(n_frames, scene, mode='default_nolure', seed=21, outliers=0.0)
    df = seq.to_df().query('likelihood > 0.5').reset_index(drop=True)
    pts3 = ref_utils.get_pairwise_3d_points_from_df(df, scene.K, scene.D.reshape((-1, 4)), scene.R, scene.t,
                                                    ref_calib.triangulate_points_fisheye, verbose=False)
    pts3['point_index'] = pts3.index
    m = df.merge(pts3, how='inner', on=['frame', 'marker'], suffixes=('_cam', ''))
    p2 = m[['x_cam', 'y_cam']].to_numpy(np.float64)
    pi = m['point_index'].to_numpy(np.int64)
    ci = m['camera'].to_numpy(np.int64)
    p3 = pts3[['x', 'y', 'z']].to_numpy(np.float64)
    # perturb the extrinsics a little so there is something to adjust
    rng = np.random.default_rng(5)
    R = scene.R.copy()
    t = scene.t.copy()
    for c in range(1, len(R)):
        rv = _cv2shim._rodrigues(R[c])[0].ravel() + rng.normal(0, 2e-3, 3)
        R[c] = _cv2shim._rodrigues(rv)[0]
        t[c] = t[c] + rng.normal(0, 5e-3, (3, 1))
    t0 = time.time()
    obj, r_out, t_out, res = ref_sba.bundle_adjust_points_and_extrinsics(
        p2, p3, pi, ci, scene.K, scene.D, R, t, ref_calib.project_points_fisheye)
    dt = time.time() - t0
    np.savez_compressed(os.path.join(HERE, 'sba_extrinsics.npz'), K=scene.K, D=scene.D, R0=R, t0=t,
                        points_2d=p2, points_3d=p3, point_indices=pi, camera_indices=ci,
                        obj_out=np.asarray(obj), R_out=np.asarray(r_out), t_out=np.asarray(t_out),
                        resid_before=np.asarray(res['before']), resid_after=np.asarray(res['after']),
                        ref_seconds=dt)
    print(f'extrinsics: {len(p2)} obs, {len(p3)} pts, ref {dt:.1f}s')


def ekf_fixture(mode='default', n_frames=30, seed=31):
    """Runs the reference's own `core.ekf.ekf` (src/core/ekf.py:26-347). Its module is
    loaded from the file with stand-ins for what it imports but does not compute with:
    pyomo / seaborn (imported, unused by the EKF), `core.metrics.save_error_dists` (plots)
    and `lib.app` (logging, the pickle/video writer and plotting); the stand-in
    `save_ekf` captures the `states` dict the reference hands to it."""
    import importlib.util
    import types
    from unittest import mock
    for name in ('pyomo', 'pyomo.environ', 'pyomo.opt', 'seaborn'):
        sys.modules.setdefault(name, mock.MagicMock())
    captured = {}
    app = types.ModuleType('lib.app')
    app.start_logging = lambda *a, **k: None
    app.stop_logging = lambda *a, **k: None
    app.plot_cheetah_states = lambda *a, **k: None

    def save_ekf(states, *a, **k):
        captured.update({key: np.asarray(v, np.float64) for key, v in states.items()})
        return 'ekf.pickle'
    app.save_ekf = save_ekf
    sys.modules['lib.app'] = app
    import lib
    lib.app = app
    core = types.ModuleType('core')
    core.__path__ = [os.path.join(REF_SRC, 'core')]
    metrics = types.ModuleType('core.metrics')
    metrics.save_error_dists = lambda *a, **k: 0.0
    sys.modules['core'] = core
    sys.modules['core.metrics'] = metrics
    spec = importlib.util.spec_from_file_location('core.ekf', os.path.join(REF_SRC, 'core', 'ekf.py'))
    ref_ekf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref_ekf)
    # the reprojection report after the smoother (ekf.py:326-333) trips over object-typed
    # columns in pandas 2 (metric.residual_error); it is not part of the fixture
    ref_ekf.metric = types.SimpleNamespace(residual_error=lambda *a, **k: {})

    scene = synth.load_scene_file()
    seq = synth.make_sequence(n_frames, scene, mode=mode, seed=seed)
    df = seq.to_df()
    cam_params = (scene.K, scene.D, scene.R, scene.t, tuple(scene.res), scene.n_cams)
    scene_path = '/tmp/golden_ekf_scene.json'
    scene.to_json(scene_path)
    out_dir = '/tmp/golden_ekf'
    os.makedirs(out_dir, exist_ok=True)
    t0 = time.time()
    ref_ekf.ekf(out_dir, df, mode, cam_params, 0, n_frames - 1, 0.5, scene_path, params={'vid_fps': 90.0})
    dt = time.time() - t0
    markers = seq.markers
    np.savez_compressed(os.path.join(HERE, f'ekf_{mode}.npz'), K=scene.K, D=scene.D, R=scene.R, t=scene.t,
                        res=np.array(scene.res), fps=90.0, thresh=0.5, n_frames=n_frames,
                        uv=seq.uv, likelihood=seq.likelihood, marker_names=np.array(markers),
                        ref_seconds=dt, **{f'out_{k}': v for k, v in captured.items()})
    print(f'ekf {mode}: {n_frames} frames, ref {dt:.1f}s, keys {sorted(captured)}')


def board_fixture(n_img=8, cams=(0, 1, 2), board_shape=(9, 6), square=0.088, seed=11):
    """Calibration-board bundle adjustment (src/lib/sba.py:37-137, :209-282): synthetic
    checkerboard corners seen by 1-3 cameras per image + hand-labelled points with NaNs,
    the reference's data preparation and its full _sba_board_points run."""
    import json
    rng = np.random.default_rng(seed)
    scene = synth.load_scene_file().subset(list(cams))
    C = scene.n_cams
    obj = ref_utils.create_board_object_pts(board_shape, square).astype(np.float64)
    obj -= obj.mean(0)
    vis_pattern = [(0, 1, 2), (0, 1), (1, 2), (0, 2), (0,), (0, 1, 2), (2,), (0, 1, 2)]
    pts_per_cam = [dict() for _ in range(C)]
    truth = {}
    for i in range(n_img):
        fn = f'img{i:05d}.jpg'
        rv = np.array([np.pi / 2, 0.0, 0.0]) + rng.normal(0, 0.25, 3)
        Rb = _cv2shim._rodrigues(rv)[0]
        ctr = np.array([1.9, 6.4, 0.6]) + rng.normal(0, 0.4, 3)
        X = obj @ Rb.T + ctr
        truth[fn] = X
        for c in vis_pattern[i % len(vis_pattern)]:
            uv = synth.project_numpy(X, scene.K[c], scene.D[c], scene.R[c], scene.t[c])
            uv = uv + rng.normal(0, 0.3, uv.shape)
            pts_per_cam[c][fn] = uv.reshape(-1, 1, 2).tolist()
    # hand-labelled points: (n_points, n_cams, 2) with NaN where a camera has no label
    n_man = 6
    Xm = np.array([1.9, 6.4, 0.5]) + rng.normal(0, 0.5, (n_man, 3))
    man = np.full((n_man, C, 2), np.nan)
    for j in range(n_man):
        for c in range(C):
            if (j + c) % 4 != 3:
                man[j, c] = synth.project_numpy(Xm[j:j + 1], scene.K[c], scene.D[c], scene.R[c], scene.t[c])[0]
    man[0, 1:] = np.nan  # seen by one camera only: dropped
    # perturbed starting extrinsics
    R0, t0 = scene.R.copy(), scene.t.copy()
    for c in range(1, C):
        R0[c] = _cv2shim._rodrigues(_cv2shim._rodrigues(R0[c])[0].ravel() + rng.normal(0, 2e-3, 3))[0]
        t0[c] = t0[c] + rng.normal(0, 5e-3, (3, 1))
    tmp = '/tmp/golden_board'
    os.makedirs(tmp, exist_ok=True)
    scene_path = os.path.join(tmp, 'scene.json')
    ref_utils.save_scene(scene_path, scene.K, scene.D, R0, t0, tuple(scene.res))
    pfs = []
    for c in range(C):
        fnames = sorted(pts_per_cam[c])
        pf = os.path.join(tmp, f'points_cam{c}.json')
        ref_utils.save_points(pf, [pts_per_cam[c][f] for f in fnames], fnames, board_shape, square, tuple(scene.res))
        pfs.append(pf)
    mf = os.path.join(tmp, 'manual_points.json')
    with open(mf, 'w') as f:
        json.dump({'points': man.tolist(), 'frame_idx': list(range(n_man)),
                   'camera_resolution': list(scene.res)}, f)
    man_loaded = ref_utils.load_manual_points(mf)[0].astype(np.float64)
    img_pts_arr, fnames_arr = [], []
    for pf in pfs:
        p, fn, *_ = ref_utils.load_points(pf)
        img_pts_arr.append(p)
        fnames_arr.append(fn)
    b2, b3, bi, bc = ref_sba.prepare_calib_board_data_for_bundle_adjustment(
        img_pts_arr, fnames_arr, board_shape, scene.K, scene.D, R0, t0, ref_calib.triangulate_points_fisheye)
    # image name of every 3-D point block (the reference walks a set: hash-seed order)
    ppi = board_shape[0] * board_shape[1]
    order = []
    for blk in range(len(b3) // ppi):
        rows = np.flatnonzero(bi == blk * ppi)[0]
        c = int(bc[rows])
        uv = b2[rows:rows + ppi]
        hit = [fn for fn, v in zip(fnames_arr[c], img_pts_arr[c]) if np.array_equal(v.reshape(-1, 2), uv)]
        order.append(hit[0])
    m2, m3, mi, mc = ref_sba.prepare_manual_points_for_bundle_adjustment(
        man_loaded, scene.K, scene.D, R0, t0, ref_calib.triangulate_points_fisheye)
    out_path = os.path.join(tmp, 'scene_sba.json')
    t_start = time.time()
    res = ref_sba._sba_board_points(scene_path, pfs, mf, out_path, ref_calib.triangulate_points_fisheye,
                                    ref_calib.project_points_fisheye)
    dt = time.time() - t_start
    _, _, R1, t1, _ = ref_utils.load_scene(out_path, verbose=False)
    files = {f'points_cam{c}': open(pfs[c]).read() for c in range(C)}
    np.savez_compressed(os.path.join(HERE, 'board.npz'), K=scene.K, D=scene.D, R_true=scene.R, t_true=scene.t,
                        R0=R0, t0=t0, res=np.array(scene.res), board_shape=np.array(board_shape), square=square,
                        manual_points_json=open(mf).read(), manual=man_loaded,
                        board_points_2d=b2, board_points_3d=b3, board_point_indices=bi, board_camera_indices=bc,
                        board_fname_order=np.array(order), manual_points_2d=m2, manual_points_3d=m3,
                        manual_point_indices=mi, manual_camera_indices=mc, R_out=R1, t_out=t1,
                        resid_before=np.asarray(res['before']), resid_after=np.asarray(res['after']),
                        ref_seconds=dt, **files)
    print(f'board: {len(b2)} board obs + {len(m2)} manual obs, ref {dt:.1f}s')


def _load_ref_fte():
    """The reference's `core.fte` module (src/core/fte.py), loaded from its file with the
    numeric Pyomo stand-in (`_pyomo_eval`) and stubs for what it imports but does not
    compute with: seaborn, `core.metrics.save_error_dists` (plots) and `lib.app`
    (logging, plots, the pickle/video writer). The stub `save_fte` captures the states
    dict the reference hands to it."""
    import importlib.util
    import types
    from unittest import mock
    import _pyomo_eval
    _pyomo_eval.install()
    sys.modules.setdefault('seaborn', mock.MagicMock())
    captured = {}
    app = types.ModuleType('lib.app')
    app.start_logging = lambda *a, **k: None
    app.stop_logging = lambda *a, **k: None
    app.plot_cheetah_states = lambda *a, **k: None
    app.plot_shutter_delay = lambda *a, **k: None

    def save_fte(states, mode, out_dir, scene_fpath, start_frame, **k):
        captured.clear()
        captured.update(states=states, start_frame=start_frame, kwargs=k)
        return os.path.join(out_dir, 'fte.pickle')
    app.save_fte = save_fte
    sys.modules['lib.app'] = app
    import lib
    lib.app = app
    core = types.ModuleType('core')
    core.__path__ = [os.path.join(REF_SRC, 'core')]
    metrics = types.ModuleType('core.metrics')
    metrics.save_error_dists = lambda *a, **k: 0.0
    sys.modules['core'] = core
    sys.modules['core.metrics'] = metrics
    spec = importlib.util.spec_from_file_location('core.fte', os.path.join(REF_SRC, 'core', 'fte.py'))
    ref_fte = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref_fte)
    return ref_fte, _pyomo_eval, captured


def fte_fixture(name, mode, n_frames, cams, sd, sd_mode, intermode, start_frame=2, seed=41, n_points=3):
    """Runs the reference's own `core.fte.fte` (src/core/fte.py:28-588) up to the IPOPT call
    and evaluates ITS model at chosen points (see `_pyomo_eval`). Recorded:

    * the reference's initial point (x, dx, ddx, poses, slack_meas, shutter delay;
      :254-292) and the triangulated nose it was fitted to;
    * which constraint blocks the reference creates (the joint-angle bounds :330-430 are
      gated on parameter names being in the MARKER list, so none is ever created);
    * `n_points` feasible points: x, dx[1], ddx[1], tau chosen at random, dx/ddx for n >= 2
      by the differences the build's elimination claims, poses / slack_meas / slack_model
      from the reference's own constraint bodies. At each: every constraint residual
      (the integration and shutter constraints must hold exactly) and the objective;
    * one infeasible point (every variable random): every constraint body and the
      objective, so each block can be restated term by term;
    * the states dict and reprojection table the reference builds from feasible point 0
      (:540-575) after the 'solve'.

    DLC rows that are not visible carry NaN in the synthetic table; they have likelihood 0
    (weight 0), and are written as 0 px here because a NaN measurement would make the
    reference's 0 * slack term NaN."""
    ref_fte, pe, captured = _load_ref_fte()
    scene = synth.load_scene_file().subset(list(cams))
    total = n_frames + start_frame + 2
    seq = synth.make_sequence(total, scene, mode=mode, seed=seed, tau_max=0.004 if sd else 0.0)
    df = seq.to_df()
    df['x'] = df['x'].fillna(0.0)
    df['y'] = df['y'].fillna(0.0)
    end_frame = start_frame + n_frames - 1
    fps = 90.0
    Ts = 1.0 / fps
    rng = np.random.default_rng(seed + 100)
    rec = {}

    nose = {}
    orig_pair = ref_fte.utils.get_pairwise_3d_points_from_df

    def pair_spy(*a, **k):
        out = orig_pair(*a, **k)
        nz = out[out['marker'] == 'nose']
        nose.update(frame=nz['frame'].to_numpy(np.float64), xyz=nz[['x', 'y', 'z']].to_numpy(np.float64))
        return out
    ref_fte.utils.get_pairwise_3d_points_from_df = pair_spy

    def evaluate(m):
        out = {}
        for cname, con in m.components(pe.Constraint).items():
            ev = con.evaluate(m)
            kinds = {v[0] for v in ev.values()}
            assert len(kinds) <= 1, (cname, kinds)
            if kinds == {'range'}:
                out[cname] = np.array([[v[1], v[2], v[3]] for v in ev.values()])
            elif ev:
                out[cname] = np.array([v[1] for v in ev.values()])
            else:
                out[cname] = np.zeros(0)
        return out, m.components(pe.Objective)['obj'].evaluate(m)

    def body_with(m, cname, vname, zero_first=None):
        """Set variable `vname` to the body of constraint `cname` evaluated with it at 0
        (the constraint's index set equals the variable's; missing indices stay 0)."""
        var = m.components(pe.Var)[vname]
        var.set_values(np.zeros(len(var.data)))
        ev = m.components(pe.Constraint)[cname].evaluate(m)
        vals = np.array([ev[k][1] if k in ev else 0.0 for k in var.keys()])
        var.set_values(vals)

    def hook(m):
        V = m.components(pe.Var)
        N, P = len(m.N), len(m.P)
        rec['init'] = {k: v.values() for k, v in V.items()}
        rec['constraints'] = sorted(m.components(pe.Constraint))
        truth = seq.x[start_frame:end_frame + 1]
        tau_shape = (N, len(cams)) if sd_mode == 'variable' else (len(cams),)
        for i in range(n_points + 1):
            x = truth + rng.normal(0, 0.02, truth.shape)
            if i < n_points:       # feasible: backward-Euler differences, constant-acc slack
                dx = np.zeros_like(x)
                ddx = np.zeros_like(x)
                dx[0] = rng.normal(0, 1.0, P)
                ddx[0] = rng.normal(0, 10.0, P)
                dx[1:] = (x[1:] - x[:-1]) / Ts
                for n in range(1, N):
                    ddx[n] = (dx[n] - dx[n - 1]) / Ts
            else:                  # infeasible: everything random
                dx = rng.normal(0, 1.0, x.shape)
                ddx = rng.normal(0, 10.0, x.shape)
            V['x'].set_values(x)
            V['dx'].set_values(dx)
            V['ddx'].set_values(ddx)
            if sd:
                tau = rng.uniform(-Ts, Ts, tau_shape)
                if i < n_points:
                    tau[..., 0] = 0.0
                V['shutter_delay'].set_values(tau)
            if i < n_points:
                body_with(m, 'pose_constraint', 'poses')
                body_with(m, 'measurement', 'slack_meas')
                body_with(m, 'constant_acc', 'slack_model')
            else:
                V['poses'].set_values(rec['init']['poses'] + rng.normal(0, 0.01, len(V['poses'].data)))
                V['slack_meas'].set_values(rng.normal(0, 5.0, len(V['slack_meas'].data)))
                V['slack_model'].set_values(rng.normal(0, 20.0, len(V['slack_model'].data)))
            cons, obj = evaluate(m)
            tag = f'pt{i}' if i < n_points else 'rand'
            rec[tag] = dict(vars={k: v.values() for k, v in V.items()}, cons=cons, obj=obj)
        # leave the model at feasible point 0 for the reference's post-processing
        for k, v in rec['pt0']['vars'].items():
            V[k].set_values(v)
        return None

    pe.SOLVE_HOOK = hook
    cam_params = (scene.K, scene.D, scene.R, scene.t, tuple(scene.res), scene.n_cams)
    scene_path = f'/tmp/golden_{name}_scene.json'
    scene.to_json(scene_path)
    out_dir = f'/tmp/golden_{name}'
    t0 = time.time()
    try:
        ref_fte.fte(out_dir, df, mode, cam_params, start_frame, end_frame, 0.5, scene_path,
                    params={'vid_fps': fps}, shutter_delay=sd, shutter_delay_mode=sd_mode,
                    interpolation_mode=intermode, video=False, plot=False)
    finally:
        ref_fte.utils.get_pairwise_3d_points_from_df = orig_pair
        pe.SOLVE_HOOK = None
    dt = time.time() - t0
    out = dict(K=scene.K, D=scene.D, R=scene.R, t=scene.t, res=np.array(scene.res), fps=fps, thresh=0.5,
               mode=mode, sd=sd, sd_mode=sd_mode, intermode=intermode, start_frame=start_frame,
               end_frame=end_frame, n_points=n_points, ref_seconds=dt, constraints=np.array(rec['constraints']),
               **_df_arrays(df, seq.markers), nose_frame=nose['frame'], nose_xyz=nose['xyz'])
    for k, v in rec['init'].items():
        out[f'init_{k}'] = v
    for tag in [f'pt{i}' for i in range(n_points)] + ['rand']:
        for k, v in rec[tag]['vars'].items():
            out[f'{tag}_var_{k}'] = v
        for k, v in rec[tag]['cons'].items():
            out[f'{tag}_con_{k}'] = v
        out[f'{tag}_obj'] = rec[tag]['obj']
    st = captured['states']
    for k in ('x', 'dx', 'ddx', 'shutter_delay'):
        if k in st:
            out[f'out_{k}'] = np.asarray(st[k], np.float64)
    errs = st.get('reprj_errors') or {}
    for c, e in errs.items():
        if e is not None and len(e):
            out[f'out_reprj_{c}'] = e[['frame', 'pixel_residual']].to_numpy(np.float64)
    out['out_start_frame'] = captured['start_frame']
    np.savez_compressed(os.path.join(HERE, f'{name}.npz'), **out)
    worst = max(float(np.abs(v).max()) for k, v in rec['pt0']['cons'].items()
                if v.size and v.ndim == 1)
    print(f'{name}: N={n_frames} C={len(cams)} mode={mode} sd={sd}/{sd_mode}/{intermode}, '
          f'constraints {rec["constraints"]}, feasible-point max |residual| {worst:.2e}, '
          f'objective {rec["pt0"]["obj"]:.6f}, reference build+eval {dt:.1f}s')


def _dlc_frames(seed, parts, n, scorer, coords=('x', 'y', 'likelihood'), str_index=False, nan_frac=0.15):
    """A synthetic DLC output table: MultiIndex columns (scorer, bodyparts, coords), rows =
    frames (int) or DLC image paths ('labeled-data/.../img0042.png')."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    cols = pd.MultiIndex.from_tuples([(scorer, bp, c) for bp in parts for c in coords],
                                     names=['scorer', 'bodyparts', 'coords'])
    v = np.empty((n, len(cols)))
    for j, (_, bp, c) in enumerate(cols):
        v[:, j] = rng.uniform(0.0, 1.0, n) if c == 'likelihood' else rng.uniform(0, 2000, n)
    # x and y go missing together mostly, alone sometimes (the reference derives a missing
    # likelihood from y in the plain branch, :111-113, and from x in the dlc_head branch, :88-91)
    miss = rng.uniform(size=(n, len(parts))) < nan_frac
    alone = rng.integers(0, 4, size=(n, len(parts)))          # 0: only x, 1: only y, else both
    for k, bp in enumerate(parts):
        for j, (_, b, c) in enumerate(cols):
            if b == bp and c in ('x', 'y'):
                drop = miss[:, k] & ((alone[:, k] >= 2) | (alone[:, k] == (0 if c == 'x' else 1)))
                v[drop, j] = np.nan
    idx = [f'labeled-data/cam/img{i + 3:04d}.png' for i in range(n)] if str_index else np.arange(n)
    return pd.DataFrame(v, index=idx, columns=cols)


def dlc_fixture():
    """`load_dlc_points_as_df` (src/lib/utils.py:77-151), the reference function itself, on
    synthetic DLC tables handed to it through a patched `pandas.read_hdf` (PyTables is not
    installed, and the reference ships no .h5 file). Cases: standard 3-coord files,
    files without a likelihood column (image-path index), the `dlc_head` branch
    (:84-103) and frame shifts (:124-135). The fixture holds each case's input tables and
    the reference's output columns."""
    import pandas as pd
    parts = ['nose', 'r_eye', 'l_eye', 'neck_base', 'spine', 'tail_base']
    cases = {
        'standard': ([_dlc_frames(1, parts, 9, 'DLC_resnet50'), _dlc_frames(2, parts, 9, 'DLC_resnet50')],
                     ['cam1DLC.h5', 'cam2DLC.h5'], None),
        'nolik': ([_dlc_frames(3, parts, 7, 'DLC_x', coords=('x', 'y'), str_index=True),
                   _dlc_frames(4, parts, 7, 'DLC_x', coords=('x', 'y'), str_index=True)],
                  ['cam1.h5', 'cam2.h5'], None),
        'shifted': ([_dlc_frames(5, parts, 8, 'DLC_resnet50') for _ in range(3)],
                    ['cam1DLC.h5', 'cam2DLC.h5', 'cam3DLC.h5'], [2, 0, -1]),
        'head': ([_dlc_frames(6 + c, ['bodypart1', 'bodypart2', 'bodypart3', 'objectA'], 6, '2019-03-09_lily_run',
                              coords=('x', 'y'), str_index=True) for c in range(2)],
                 ['/data/dlc_head/cam1.h5', '/data/dlc_head/cam2.h5'], None),
    }
    out = {}
    orig = pd.read_hdf
    for name, (tables, paths, shifts) in cases.items():
        by_path = dict(zip(paths, tables))
        pd.read_hdf = lambda p, *a, **k: by_path[p].copy()
        try:
            ref = ref_utils.load_dlc_points_as_df(paths, frame_shifts=shifts)
        finally:
            pd.read_hdf = orig
        for c, (p, t) in enumerate(zip(paths, tables)):
            out[f'{name}_in{c}_values'] = t.to_numpy(np.float64)
            out[f'{name}_in{c}_columns'] = np.array(['|'.join(col) for col in t.columns])
            out[f'{name}_in{c}_index'] = np.array([str(s) for s in t.index])
            out[f'{name}_in{c}_int_index'] = np.array(not isinstance(t.index[0], str))
            out[f'{name}_in{c}_path'] = np.array(p)
        out[f'{name}_ncams'] = np.array(len(paths))
        out[f'{name}_shifts'] = np.array(shifts if shifts is not None else [], np.int64)
        out[f'{name}_out_frame'] = np.array([str(f) for f in ref['frame']])
        out[f'{name}_out_camera'] = ref['camera'].to_numpy(np.int64)
        out[f'{name}_out_marker'] = np.array([str(m) for m in ref['marker']])
        for k in ('x', 'y', 'likelihood'):
            out[f'{name}_out_{k}'] = ref[k].to_numpy(np.float64)
        print(f'dlc {name}: {len(ref)} rows, cams {len(paths)}, shifts {shifts}')
    np.savez_compressed(os.path.join(HERE, 'dlc.npz'), **out)


def _load_ref_app_and_tri():
    """The reference's `lib.app` (src/lib/app.py) and `core.tri` (src/core/tri.py), loaded
    from their files. Stand-ins only for what they import but do not compute with on this
    path: `lib.plotting` / `lib.vid` / `lib.points` (GUI, video, checkerboard detection),
    pyomo / seaborn (imported by core.tri, unused) and `core.metrics.save_error_dists`
    (PDF histograms; it also fails on residual_error's string columns).
    `create_labeled_videos` is replaced by a no-op (rendering)."""
    import importlib.util
    import types
    from unittest import mock
    for name in ('pyomo', 'pyomo.environ', 'pyomo.opt', 'seaborn', 'lib.plotting', 'lib.vid', 'lib.points'):
        sys.modules[name] = mock.MagicMock()
    import lib
    spec = importlib.util.spec_from_file_location('lib.app', os.path.join(REF_SRC, 'lib', 'app.py'))
    ref_app = importlib.util.module_from_spec(spec)
    sys.modules['lib.app'] = ref_app
    spec.loader.exec_module(ref_app)
    lib.app = ref_app
    ref_app.create_labeled_videos = lambda *a, **k: None
    core = types.ModuleType('core')
    core.__path__ = [os.path.join(REF_SRC, 'core')]
    metrics = types.ModuleType('core.metrics')
    metrics.save_error_dists = lambda *a, **k: 0.0
    sys.modules['core'] = core
    sys.modules['core.metrics'] = metrics
    spec = importlib.util.spec_from_file_location('core.tri', os.path.join(REF_SRC, 'core', 'tri.py'))
    ref_tri = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref_tri)
    return ref_app, ref_tri


class _HdfCapture:
    """`DataFrame.to_hdf` needs PyTables (absent): capture (path, key, frame) instead."""

    def __init__(self):
        import pandas as pd
        self.pd = pd
        self.frames = []

    def __enter__(self):
        self.orig = self.pd.DataFrame.to_hdf
        frames = self.frames

        def to_hdf(df, path, key, *a, **k):
            frames.append((os.path.basename(path), key, df.copy()))
        self.pd.DataFrame.to_hdf = to_hdf
        return self

    def __exit__(self, *exc):
        self.pd.DataFrame.to_hdf = self.orig


def _frame_arrays(prefix, frames, out_dir, out):
    """Per camera: values (n_frames, 3 L), index, column tuples, and the CSV text the
    reference wrote beside the (captured) .h5."""
    out[f'{prefix}_n'] = np.array(len(frames))
    for i, (fname, key, df) in enumerate(frames):
        out[f'{prefix}{i}_fname'] = np.array(fname)
        out[f'{prefix}{i}_key'] = np.array(key)
        out[f'{prefix}{i}_values'] = df.to_numpy(np.float64)
        out[f'{prefix}{i}_index'] = df.index.to_numpy(np.int64)
        out[f'{prefix}{i}_columns'] = np.array(['|'.join(c) for c in df.columns])
        out[f'{prefix}{i}_col_names'] = np.array([str(n) for n in df.columns.names])
        with open(os.path.join(out_dir, os.path.splitext(fname)[0] + '.csv')) as f:
            out[f'{prefix}{i}_csv'] = np.array(f.read())


def save2d_tri_fixture(n_frames=12, seed=53):
    """`save_3d_cheetah_as_2d` (src/lib/utils.py:237-286) and `core.tri` + `app.save_tri`
    (src/core/tri.py:27-64, src/lib/app.py:238-268), the reference functions themselves.

    * tri: a 6-camera synthetic sequence (20 keypoints + NaN rows) through the reference's
      `core.tri` with cam1..6.mp4 beside the output: tri.pickle's contents (captured at
      `utils.save_optimised_cheetah`), and the cam*_tri frames / CSVs.
    * save2d: per-camera position lists (FTE style: one array per camera) with NaN points,
      points outside the image and points behind a camera, projected by the reference
      into cam*_fte frames; also the single-array (SBA / EKF) form with `out_fname`."""
    import pandas as pd
    ref_app, ref_tri = _load_ref_app_and_tri()
    root = '/tmp/golden_save2d'
    import shutil
    shutil.rmtree(root, ignore_errors=True)
    data_dir = os.path.join(root, 'data', '2019_03_09', 'run')
    calib_dir = os.path.join(root, 'data', '2019_03_09', 'extrinsic_calib')
    os.makedirs(data_dir)
    os.makedirs(calib_dir)
    scene = synth.load_scene_file()
    C = scene.n_cams
    scene_path = os.path.join(calib_dir, f'{C}_cam_scene_sba.json')
    scene.to_json(scene_path)
    for c in range(C):
        open(os.path.join(data_dir, f'cam{c + 1}.mp4'), 'wb').close()
    seq = synth.make_sequence(n_frames, scene, mode='default_nolure', seed=seed)
    start_frame = 3
    df = seq.to_df(start_frame=start_frame)
    df = df[np.isfinite(df['x']) & np.isfinite(df['y'])].reset_index(drop=True)
    out = dict(K=scene.K, D=scene.D, R=scene.R, t=scene.t, res=np.array(scene.res), n_frames=n_frames,
               start_frame=start_frame, thresh=0.5, marker_names=np.array(seq.markers),
               **_df_arrays(df, seq.markers))

    # --- core.tri -> app.save_tri -> utils.save_3d_cheetah_as_2d
    cap = {}
    orig_save = ref_tri.utils.save_optimised_cheetah

    def save_spy(positions, out_fpath, extra_data=None, **k):
        cap.update(positions=np.array(positions, np.float64), fname=os.path.basename(out_fpath),
                   extra=dict(extra_data or {}))
    ref_tri.utils.save_optimised_cheetah = save_spy
    cam_params = (scene.K, scene.D, scene.R, scene.t, tuple(scene.res), C)
    try:
        with _HdfCapture() as hc:
            fp = ref_tri.tri(data_dir, df, start_frame, start_frame + n_frames - 1, 0.5, cam_params, scene_path)
    finally:
        ref_tri.utils.save_optimised_cheetah = orig_save
    out['tri_out_fname'] = np.array(os.path.relpath(fp, data_dir))
    out['tri_positions'] = cap['positions']
    out['tri_pickle_fname'] = np.array(cap['fname'])
    out['tri_start_frame'] = np.array(cap['extra']['start_frame'])
    out['tri_extra_keys'] = np.array(sorted(cap['extra']))
    tri_markers = ref_misc.get_markers(mode='all') + ['coe', 'gaze_target']
    out['tri_markers'] = np.array(tri_markers)
    for c, e in cap['extra']['errors'].items():
        out[f'tri_err{c}'] = e[['frame', 'camera_distance', 'pixel_residual', 'pck_threshold', 'error_u',
                               'error_v']].to_numpy().astype(np.float64)
        out[f'tri_err{c}_marker'] = e['marker'].to_numpy().astype(str)
    with open(os.path.join(data_dir, 'tri', 'reconstruction_params.json')) as f:
        out['tri_params_json'] = np.array(f.read())
    _frame_arrays('tri2d', hc.frames, os.path.join(data_dir, 'tri'), out)

    # --- save_3d_cheetah_as_2d, FTE-style list of per-camera arrays
    rng = np.random.default_rng(seed + 7)
    fte_dir = os.path.join(data_dir, 'fte')
    os.makedirs(fte_dir)
    L2 = 5
    bodyparts = ['nose', 'r_eye', 'l_eye', 'coe', 'gaze_target']
    pos = []
    for c in range(C):
        p = np.array([1.9, 6.4, 0.6]) + rng.normal(0, 0.4, (n_frames, L2, 3))
        p[rng.random((n_frames, L2)) < 0.1] = np.nan                      # missing points
        p[0, 1] = [1.9, 6.4, 40.0]                                        # far above: outside the image
        p[1, 2] = (-scene.R[c].T @ scene.t[c]).ravel() - 0.5 * scene.R[c][2]  # behind camera c
        p[2, 0] = [1.9 + 30.0 * (c % 2), 6.4 - 30.0 * (c // 3), 0.6]        # wide angle
        pos.append(p)
    with _HdfCapture() as hc:
        ref_utils.save_3d_cheetah_as_2d(pos, fte_dir, scene_path, list(bodyparts), ref_calib.project_points_fisheye,
                                        start_frame)
    out['fte_pos'] = np.array(pos)
    out['fte_bodyparts'] = np.array(bodyparts)
    _frame_arrays('fte2d', hc.frames, fte_dir, out)

    # --- single array (save_sba / save_ekf form), out_fname given, no CSV
    with _HdfCapture() as hc:
        ref_utils.save_3d_cheetah_as_2d(pos[0], fte_dir, scene_path, list(bodyparts), ref_calib.project_points_fisheye,
                                        start_frame, save_as_csv=False, out_fname='custom')
    out['one_n'] = np.array(len(hc.frames))
    for i, (fname, key, d) in enumerate(hc.frames):
        out[f'one{i}_fname'] = np.array(fname)
        out[f'one{i}_key'] = np.array(key)
        out[f'one{i}_values'] = d.to_numpy(np.float64)
    np.savez_compressed(os.path.join(HERE, 'save2d_tri.npz'), **out)
    print(f'save2d_tri: tri {cap["positions"].shape}, {len(out["fte_pos"])} cameras of fte-style projections')


if __name__ == '__main__':
    which = sys.argv[1:] or ['loss', 'fk', 'tri', 'cfg1', 'cfg2', 'ext']
    if 'save2d' in which:
        save2d_tri_fixture()
    if 'dlc' in which:
        dlc_fixture()
    if 'fte' in which:
        fte_fixture('fte_head_const', 'head', 8, range(6), True, 'const', 'vel')
        fte_fixture('fte_default_const', 'default', 5, range(6), True, 'const', 'vel')
        fte_fixture('fte_default_var_acc', 'default', 4, range(3), True, 'variable', 'acc')
        fte_fixture('fte_head_nosd', 'head', 6, range(3), False, 'const', 'pos')
    if 'loss' in which:
        loss_fixture()
    if 'fk' in which:
        fk_fixture()
    if 'tri' in which:
        triangulation_fixture()
    if 'cfg1' in which:
        sba_fixture('sba_cfg1', 10, [0, 1])
    if 'cfg2' in which:
        sba_fixture('sba_cfg2', 100, list(range(6)))
    if 'ext' in which:
        extrinsics_fixture()
    if 'board' in which:
        board_fixture()
    if 'ekf' in which:
        ekf_fixture('default', 30)
        ekf_fixture('head', 40)
