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


def _dlc_csv(path, parts, n, seed, likelihood=True, str_index=False):
    """A DLC-style export: 3 header rows (scorer / bodyparts / coords), one row per frame."""
    rng = np.random.default_rng(seed)
    coords = ['x', 'y', 'likelihood'] if likelihood else ['x', 'y']
    cols = pd.MultiIndex.from_product([['DLC_resnet50_cheetahOct1shuffle1_200000'], parts, coords],
                                      names=['scorer', 'bodyparts', 'coords'])
    v = rng.uniform(0, 1000, (n, len(cols)))
    v[rng.random(v.shape) < 0.05] = np.nan
    idx = [f'labeled-data/run/img{k:03d}.png' for k in range(n)] if str_index else np.arange(n)
    df = pd.DataFrame(v, index=idx, columns=cols)
    df.to_csv(path)
    return df


def _expected_long(df, cam, shift):
    """Row-by-row restatement of src/lib/utils.py:77-151 on one file: markers in sorted order
    within a frame (the `.T.unstack().T` reshape sorts the bodyparts level, :115), rows moved
    by `shift` frames with NaN / likelihood 0 shifted in (:118-132), frame column unshifted."""
    d = df.droplevel(0, axis=1)
    parts = sorted(set(d.columns.get_level_values(0)))
    has_lk = 'likelihood' in set(d.columns.get_level_values(1))
    n = len(d)
    frames = [int(str(s)[-7:-4]) if isinstance(s, str) else int(s) for s in d.index]
    rows = []
    for k in range(n):
        src = k - shift
        for bp in parts:
            if 0 <= src < n:
                x, y = d[(bp, 'x')].iloc[src], d[(bp, 'y')].iloc[src]
                lk = d[(bp, 'likelihood')].iloc[src] if has_lk else (0.0 if np.isnan(x) else 1.0)
            else:
                x = y = lk = np.nan
            rows.append((frames[k], cam, bp, x, y, 0.0 if np.isnan(lk) else lk))
    return pd.DataFrame(rows, columns=['frame', 'camera', 'marker', 'x', 'y', 'likelihood'])


@pytest.mark.parametrize('shifts', [None, [0, 2, -3]])
def test_load_dlc_points_as_df_matches_reference_reshape(tmp_path, shifts):
    from acinoset_amd.lib import utils as lu
    parts = ['nose', 'r_eye', 'l_eye', 'neck_base', 'tail_tip']
    paths, dfs = [], []
    for c in range(3):
        p = str(tmp_path / f'cam{c + 1}DLC.csv')
        dfs.append(_dlc_csv(p, parts, 12, seed=c, likelihood=(c != 1), str_index=(c == 2)))
        paths.append(p)
    got = lu.load_dlc_points_as_df(paths, frame_shifts=shifts)
    exp = pd.concat([_expected_long(df, c, 0 if shifts is None else shifts[c]) for c, df in enumerate(dfs)],
                    ignore_index=True)
    assert list(got.columns) == ['frame', 'camera', 'marker', 'x', 'y', 'likelihood']
    assert got[['frame', 'camera', 'marker']].astype(str).equals(exp[['frame', 'camera', 'marker']].astype(str))
    for col in ('x', 'y', 'likelihood'):
        np.testing.assert_allclose(got[col].to_numpy(float), exp[col].to_numpy(float), rtol=0, atol=1e-9,
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
