"""CPU: host-side glue of the drop-in layer (no GPU calls)."""
import pytest
import numpy as np
import pandas as pd

from oracle import fte as ofte
from acinoset_amd import synth
import importlib
cfte = importlib.import_module("acinoset_amd.core.fte")
from acinoset_amd.kinematics import get_markers


def test_build_measurements_matches_reference_lookup():
    seq = synth.make_sequence(6, synth.load_scene_file(), mode='head', seed=1)
    df = seq.to_df(start_frame=10)
    markers = get_markers('head')
    meas, w = cfte.build_measurements(df, markers, 6, 11, 14, 0.5)
    # reference semantics (src/core/fte.py:195-221): boolean-mask lookup, first row
    for n in range(4):
        for c in range(6):
            for l, m in enumerate(markers):
                row = df[(df['frame'] == n + 11) & (df['marker'] == m) & (df['camera'] == c)]
                lk = row['likelihood'].values[0]
                assert w[n, c, l] == (1 / 3 if lk > 0.5 else 0.0)
                if np.isfinite(row['x'].values[0]):
                    assert meas[n, c, l, 0] == row['x'].values[0] and meas[n, c, l, 1] == row['y'].values[0]


def test_initial_state_matches_reference_linregress():
    rng = np.random.default_rng(0)
    fr = np.arange(5, 45)
    xyz = np.stack([1 + 0.05 * fr, 6 - 0.01 * fr, 0.6 + 0 * fr], 1) + rng.normal(0, 0.01, (40, 3))
    df = pd.DataFrame({'frame': fr, 'marker': 'nose', 'x': xyz[:, 0], 'y': xyz[:, 1], 'z': xyz[:, 2]})
    X = cfte.initial_state(df, 'default_nolure', 5, 44)
    prob = type('P', (), {'mode': 'default_nolure', 'N': 40, 'P': 26})()
    Xo = ofte.initial_state(prob, fr, xyz, start_frame=5)
    np.testing.assert_allclose(X, Xo, atol=1e-12)


def test_states_satisfy_reference_integration_constraints():
    """x_n = x_{n-1} + Ts dx_n, dx_n = dx_{n-1} + Ts ddx_n for n >= 2 (src/core/fte.py:467-477)."""
    rng = np.random.default_rng(1)
    X = rng.normal(size=(12, 6))
    Ts = 1 / 90
    st = cfte.states_from_solution(X, np.array([0.0, 1e-3]), Ts, True, 10)
    x, dx, ddx = (np.asarray(st[k]) for k in ('x', 'dx', 'ddx'))
    np.testing.assert_allclose(x[1:], x[:-1] + Ts * dx[1:], atol=1e-12)
    np.testing.assert_allclose(dx[1:], dx[:-1] + Ts * ddx[1:], atol=1e-9)
    assert len(st['shutter_delay']) == 2 and len(st['shutter_delay'][1]) == 10


def test_model_weights_are_reference_Q():
    q = cfte.model_weights('head')
    np.testing.assert_allclose(q, 1 / np.array([4, 7, 5, 13, 9, 26], float) ** 2)


def test_ekf_model_matrices_match_oracle():
    """P0 / Q / R std of the drop-in (acinoset_amd.core.ekf) equal the oracle restatement of
    src/core/ekf.py:159-213."""
    import importlib
    from oracle import ekf as oekf
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    for mode, P in (('default', 29), ('head', 6)):
        np.testing.assert_array_equal(cekf.initial_covariance(mode), oekf.initial_covariance(mode))
        np.testing.assert_array_equal(cekf.process_covariance(P, 1 / 90.0), oekf.process_noise(P, 1 / 90.0))
    np.testing.assert_allclose(cekf.measurement_std(6), [2 * c / 0.087 for c in oekf.CAL_COVS])
    assert cekf.initial_covariance('default')[6, 6] == -0.28   # the reference's neck-length entry


def test_ekf_initial_state_matches_oracle():
    import importlib
    import pandas as pd
    from conftest import golden
    from oracle import ekf as oekf, fisheye
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    g = golden('ekf_default')
    N = int(g['n_frames'])
    uv = g['uv']
    C, L = uv.shape[1], uv.shape[2]
    fr, ca, mk = np.meshgrid(np.arange(N), np.arange(C), np.arange(L), indexing='ij')
    fr_, mk_, xyz = fisheye.pairwise_points(fr.ravel(), ca.ravel(), mk.ravel(), uv[..., 0].ravel(),
                                            uv[..., 1].ravel(), g['K'], g['D'], g['R'], g['t'])
    names = list(g['marker_names'])
    df = pd.DataFrame({'frame': fr_, 'marker': [names[m] for m in mk_], 'x': xyz[:, 0], 'y': xyz[:, 1],
                       'z': xyz[:, 2]})
    np.testing.assert_allclose(cekf.initial_state(df, 'default', 0, 90.0),
                               oekf.initial_state('default', fr_, mk_, xyz, 0, 1 / 90.0), rtol=1e-10, atol=1e-10)


def test_ekf_dense_observations_pivot():
    import importlib
    from acinoset_amd import synth
    cekf = importlib.import_module('acinoset_amd.core.ekf')
    seq = synth.make_sequence(5, synth.load_scene_file(), mode='head', seed=1)
    df = seq.to_df()
    df = df.drop(index=[0, 7]).reset_index(drop=True)           # two missing rows -> NaN
    meas, lik = cekf.dense_observations(df, seq.markers, 6, 5)
    assert np.isnan(meas).sum() == 4 and np.isnan(lik).sum() == 2
    ok = ~np.isnan(lik)
    np.testing.assert_array_equal(lik[ok], seq.likelihood[ok])
    np.testing.assert_array_equal(meas[ok], seq.uv[ok])


def test_states_variable_shutter_delay_layout():
    """variable mode: sd_state = [[tau[n, c] for n] for c] (src/core/fte.py:553-554)."""
    X = np.zeros((7, 6))
    tau = np.arange(15.0).reshape(5, 3) * 1e-4
    st = cfte.states_from_solution(X, tau, 1 / 90, True, 5)
    assert np.array_equal(np.asarray(st['shutter_delay']), tau.T)


@pytest.mark.parametrize('name', ['standard', 'shifted'])
def test_load_dlc_csv_route_matches_reference(tmp_path, name):
    """DLC's .csv export of the same tables (the route on boxes without PyTables) gives what
    the reference function made of the .h5 tables (tests/golden/dlc.npz)."""
    from acinoset_amd.lib import utils as lu
    from tests.test_dlc_reference import GOLD, _inputs
    d = np.load(GOLD)
    tables, paths, shifts = _inputs(d, name)
    csvs = []
    for k, p in enumerate(paths):
        q = str(tmp_path / f'cam{k + 1}DLC.csv')
        tables[p].to_csv(q)
        csvs.append(q)
    got = lu.load_dlc_points_as_df(csvs, frame_shifts=shifts)
    np.testing.assert_array_equal(np.array([str(f) for f in got['frame']]), d[f'{name}_out_frame'])
    np.testing.assert_array_equal(np.array([str(m) for m in got['marker']]), d[f'{name}_out_marker'])
    for col in ('x', 'y', 'likelihood'):
        np.testing.assert_allclose(got[col].to_numpy(float), d[f'{name}_out_{col}'], rtol=0, atol=1e-9,
                                   equal_nan=True)


def _reference_frame_range(filtered, target_markers):
    """`src/all_optimizations.py:79-111` as written: one query per frame."""
    def frame_condition(i):
        cond = ' or '.join([f'marker=="{ref}"' for ref in target_markers])
        return len(filtered.query(f'frame == {i} and ({cond})')['marker'].unique()) >= len(target_markers)
    start, end = None, None
    max_idx = int(filtered['frame'].max() + 1)
    for i in range(max_idx):
        if frame_condition(i):
            start = i
            break
    for i in range(max_idx, 0, -1):
        if frame_condition(i):
            end = i
            break
    return start, end


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_all_optimizations_frame_range_matches_reference(seed):
    from acinoset_amd import all_optimizations as ao
    rng = np.random.default_rng(seed)
    seq = synth.make_sequence(30, synth.load_scene_file(), mode='head', seed=seed)
    df = seq.to_df(start_frame=3)
    lik = df['likelihood'].to_numpy().copy()
    # whole frames without some marker at the start and the end, random dropouts elsewhere
    f = df['frame'].to_numpy()
    lik[(f < 3 + 2 + seed) & (df['marker'].to_numpy() == 'nose')] = 0.0
    lik[(f > 3 + 25 - seed) & (df['marker'].to_numpy() == 'r_eye')] = 0.0
    lik[rng.random(len(lik)) < 0.5] = 0.0
    df['likelihood'] = lik
    filt = df.query('likelihood > 0.8')
    assert ao.auto_frame_range(filt, get_markers('head')) == _reference_frame_range(filt, get_markers('head'))


def test_sparsity_pattern_metadata():
    """`create_bundle_adjustment_jacobian_sparsity_matrix` (src/lib/sba.py:11-22): rows 2i,
    2i+1 touch observation i's camera block and its point's 3 columns, [cameras | points]."""
    from acinoset_amd.lib.sba import create_bundle_adjustment_jacobian_sparsity_matrix as sparsity
    rng = np.random.default_rng(5)
    n_cams, n_pts, n_obs, pc = 4, 7, 25, 6
    cam = rng.integers(0, n_cams, n_obs)
    pt = rng.integers(0, n_pts, n_obs)
    A = sparsity(n_cams, pc, cam, n_pts, pt)
    D = np.zeros((2 * n_obs, n_cams * pc + 3 * n_pts), int)
    for i in range(n_obs):
        for r in (2 * i, 2 * i + 1):
            D[r, cam[i] * pc:(cam[i] + 1) * pc] = 1
            D[r, n_cams * pc + 3 * pt[i]:n_cams * pc + 3 * pt[i] + 3] = 1
    assert A.shape == D.shape
    np.testing.assert_array_equal(A.toarray(), D)
    assert sparsity(n_cams, 0, cam, n_pts, pt).shape == (2 * n_obs, 3 * n_pts)
