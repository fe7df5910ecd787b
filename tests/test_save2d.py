"""2-D reprojection export (`save_3d_cheetah_as_2d`, src/lib/utils.py:237-286) and the
`core.tri` / `app.save_tri` drop-in (src/core/tri.py:27-64, src/lib/app.py:238-268),
against the reference functions' own outputs (`tests/golden/save2d_tri.npz`, written by
`make_golden.py save2d` with `DataFrame.to_hdf` captured: PyTables is absent).

CPU tests here: the host logic (directory search, out-of-image rule, DLC column layout,
CSV text) with the oracle projection handed in as `project_func` (the function takes
any callable with the reference's signature). GPU tests: the same through the GPU
projection, and `core.tri` end to end."""
import io
import os
import pickle

import numpy as np
import pandas as pd
import pytest

from conftest import golden
from acinoset_amd import kinematics as pkin
from acinoset_amd.lib import utils

MARKERS20 = pkin.get_markers('default_nolure')


def _layout(g, tmp_path):
    """data/<date>/run/cam1..C.mp4 and data/<date>/extrinsic_calib/<C>_cam_scene_sba.json,
    as the reference's directory convention (and the fixture run) has them."""
    run = os.path.join(tmp_path, 'data', '2019_03_09', 'run')
    calib = os.path.join(tmp_path, 'data', '2019_03_09', 'extrinsic_calib')
    os.makedirs(run)
    os.makedirs(calib)
    C = len(g['K'])
    scene = os.path.join(calib, f'{C}_cam_scene_sba.json')
    utils.save_scene(scene, g['K'], g['D'], g['R'], g['t'], [int(v) for v in g['res']])
    for c in range(C):
        open(os.path.join(run, f'cam{c + 1}.mp4'), 'wb').close()
    return run, scene


def _oracle_project(pts, k, d, r, t):
    from oracle import fisheye
    return fisheye.project(np.asarray(pts, np.float64).reshape(-1, 3), k, d, r, t)


def _read_csv(text):
    return pd.read_csv(io.StringIO(text), header=[0, 1], index_col=0)


def check_frames(dfs, g, prefix, out_dir, atol):
    n = int(g[f'{prefix}_n'])
    assert len(dfs) == n
    for i, df in enumerate(dfs):
        ref = g[f'{prefix}{i}_values']
        got = df.to_numpy(np.float64)
        assert got.shape == ref.shape
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        np.testing.assert_allclose(got, ref, rtol=0, atol=atol, equal_nan=True)
        np.testing.assert_array_equal(df.index.to_numpy(), g[f'{prefix}{i}_index'])
        assert ['|'.join(c) for c in df.columns] == list(g[f'{prefix}{i}_columns'])
        assert [str(nm) for nm in df.columns.names] == list(g[f'{prefix}{i}_col_names'])
        csv_name = os.path.splitext(str(g[f'{prefix}{i}_fname']))[0] + '.csv'
        with open(os.path.join(out_dir, csv_name)) as f:
            text = f.read()
        ref_text = str(g[f'{prefix}{i}_csv'])
        # same header rows and row labels; values to the tolerance
        assert text.splitlines()[:2] == ref_text.splitlines()[:2]
        a, b = _read_csv(text), _read_csv(ref_text)
        np.testing.assert_array_equal(a.index, b.index)
        np.testing.assert_allclose(a.to_numpy(np.float64), b.to_numpy(np.float64), rtol=0, atol=atol,
                                   equal_nan=True)


def _save2d(g, tmp_path, project):
    run, scene = _layout(g, tmp_path)
    out_dir = os.path.join(run, 'fte')
    os.makedirs(out_dir)
    pos = [p for p in g['fte_pos']]
    dfs = utils.save_3d_cheetah_as_2d(pos, out_dir, scene, list(g['fte_bodyparts']), project,
                                      int(g['start_frame']))
    return dfs, out_dir, run, scene


def test_save2d_host_logic_matches_reference(tmp_path):
    """Oracle projection: everything but the projection is the drop-in's own logic."""
    g = golden('save2d_tri')
    dfs, out_dir, run, scene = _save2d(g, tmp_path, _oracle_project)
    check_frames(dfs, g, 'fte2d', out_dir, atol=1e-9)
    # out-of-image rule: some points are NaN only because they fall outside the image
    vals = np.stack([d.to_numpy() for d in dfs])
    assert np.isnan(vals[..., 0::3]).sum() > np.isnan(g['fte_pos'][..., 0]).sum()


def test_save2d_single_array_and_out_fname(tmp_path):
    g = golden('save2d_tri')
    run, scene = _layout(g, tmp_path)
    out_dir = os.path.join(run, 'fte')
    os.makedirs(out_dir)
    dfs = utils.save_3d_cheetah_as_2d(g['fte_pos'][0], out_dir, scene, list(g['fte_bodyparts']), _oracle_project,
                                      int(g['start_frame']), save_as_csv=False, out_fname='custom')
    assert len(dfs) == int(g['one_n'])
    for i, df in enumerate(dfs):
        np.testing.assert_allclose(df.to_numpy(np.float64), g[f'one{i}_values'], rtol=0, atol=1e-9, equal_nan=True)
        assert os.path.exists(os.path.join(out_dir, f'cam{i + 1}_custom.csv')) or \
            os.path.exists(os.path.join(out_dir, f'cam{i + 1}_custom.h5'))


def test_save2d_no_videos_and_scene_check(tmp_path):
    g = golden('save2d_tri')
    run, scene = _layout(g, tmp_path)
    for c in range(len(g['K'])):
        os.remove(os.path.join(run, f'cam{c + 1}.mp4'))
    out_dir = os.path.join(run, 'fte')
    os.makedirs(out_dir)
    assert utils.save_3d_cheetah_as_2d(g['fte_pos'][0], out_dir, scene, list(g['fte_bodyparts']),
                                       _oracle_project, 0) == []
    with pytest.raises(AssertionError):
        utils.save_3d_cheetah_as_2d(g['fte_pos'][0], '/elsewhere/fte', scene, list(g['fte_bodyparts']),
                                    _oracle_project, 0)


def _tri_df(g):
    return pd.DataFrame({'frame': g['df_frame'], 'camera': g['df_camera'],
                         'marker': np.array(MARKERS20, dtype=object)[g['df_marker']],
                         'x': g['df_x'], 'y': g['df_y'], 'likelihood': g['df_likelihood']})


@pytest.mark.gpu
def test_save2d_gpu_projection_matches_reference(tmp_path):
    from acinoset_amd.lib import calib
    g = golden('save2d_tri')
    dfs, out_dir, _, _ = _save2d(g, tmp_path, calib.project_points_fisheye)
    check_frames(dfs, g, 'fte2d', out_dir, atol=1e-9)


@pytest.mark.gpu
def test_core_tri_matches_reference(tmp_path):
    """core.tri on the GPU triangulation: tri.pickle (positions with coe / gaze target,
    start_frame, per-camera error tables), reconstruction_params.json and the cam*_tri
    reprojections, against the reference's core.tri on the same table."""
    from acinoset_amd import core
    g = golden('save2d_tri')
    run, scene = _layout(g, tmp_path)
    s0 = int(g['start_frame'])
    n = int(g['n_frames'])
    cp = (g['K'], g['D'], g['R'], g['t'], tuple(int(v) for v in g['res']), len(g['K']))
    out = core.tri(run, _tri_df(g), s0, s0 + n - 1, float(g['thresh']), cp, scene)
    assert os.path.relpath(out, run) == str(g['tri_out_fname'])
    with open(out, 'rb') as f:
        data = pickle.load(f)
    assert sorted(k for k in data if k != 'positions') == list(g['tri_extra_keys'])
    assert data['start_frame'] == int(g['tri_start_frame'])
    ref = g['tri_positions']
    np.testing.assert_array_equal(np.isnan(data['positions']), np.isnan(ref))
    np.testing.assert_allclose(data['positions'], ref, rtol=0, atol=1e-9, equal_nan=True)
    for c, e in data['errors'].items():
        cols = ['frame', 'camera_distance', 'pixel_residual', 'pck_threshold', 'error_u', 'error_v']
        np.testing.assert_allclose(e[cols].to_numpy(np.float64), g[f'tri_err{c}'], rtol=0, atol=1e-7)
        assert list(e['marker']) == list(g[f'tri_err{c}_marker'])
    with open(os.path.join(run, 'tri', 'reconstruction_params.json')) as f:
        assert f.read() == str(g['tri_params_json'])
    dfs = [pd.read_csv(os.path.join(run, 'tri', f'cam{c + 1}_tri.csv'), header=[0, 1], index_col=0)
           for c in range(len(g['K']))]
    # positions agree to 1e-9 m: their projections to 1e-6 px
    check_frames(dfs, g, 'tri2d', os.path.join(run, 'tri'), atol=1e-6)
