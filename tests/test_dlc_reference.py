"""DLC ingestion pinned to the reference function itself.

`tests/golden/dlc.npz` holds synthetic DLC tables and what the reference's own
`load_dlc_points_as_df` (src/lib/utils.py:77-151) made of them, run by
`tests/golden/make_golden.py dlc` with `pandas.read_hdf` handing the tables over (PyTables
is absent). Cases: standard files, files without a likelihood column, the `dlc_head`
branch and frame shifts. The drop-in must return the same rows in the same order.
"""
import os

import numpy as np
import pandas as pd
import pytest

from acinoset_amd.lib import utils as lu

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'dlc.npz')
CASES = ('standard', 'nolik', 'shifted', 'head')


def _inputs(d, name):
    tables, paths = {}, []
    for c in range(int(d[f'{name}_ncams'])):
        cols = pd.MultiIndex.from_tuples([tuple(s.split('|')) for s in d[f'{name}_in{c}_columns']],
                                         names=['scorer', 'bodyparts', 'coords'])
        idx = d[f'{name}_in{c}_index']
        idx = idx.astype(np.int64) if bool(d[f'{name}_in{c}_int_index']) else list(idx)
        p = str(d[f'{name}_in{c}_path'])
        tables[p] = pd.DataFrame(d[f'{name}_in{c}_values'], index=idx, columns=cols)
        paths.append(p)
    shifts = d[f'{name}_shifts']
    return tables, paths, (list(shifts) if len(shifts) else None)


@pytest.mark.parametrize('name', CASES)
def test_load_dlc_points_matches_reference(monkeypatch, name):
    d = np.load(GOLD)
    tables, paths, shifts = _inputs(d, name)
    monkeypatch.setattr(lu, '_read_dlc', lambda p: tables[p].copy())
    got = lu.load_dlc_points_as_df(paths, frame_shifts=shifts)
    assert list(got.columns) == ['frame', 'camera', 'marker', 'x', 'y', 'likelihood']
    assert len(got) == len(d[f'{name}_out_x'])
    np.testing.assert_array_equal(np.array([str(f) for f in got['frame']]), d[f'{name}_out_frame'])
    np.testing.assert_array_equal(got['camera'].to_numpy(np.int64), d[f'{name}_out_camera'])
    np.testing.assert_array_equal(np.array([str(m) for m in got['marker']]), d[f'{name}_out_marker'])
    for k in ('x', 'y', 'likelihood'):
        np.testing.assert_array_equal(got[k].to_numpy(np.float64), d[f'{name}_out_{k}'], err_msg=k)


def test_dlc_head_branch_keys_on_first_path(monkeypatch):
    """The reference tests only dlc_df_fpaths[0] for 'dlc_head' (:84): a head file listed
    second is read as a plain file."""
    d = np.load(GOLD)
    tables, paths, _ = _inputs(d, 'standard')
    monkeypatch.setattr(lu, '_read_dlc', lambda p: tables[p].copy())
    got = lu.load_dlc_points_as_df(paths)
    assert set(got['marker']) == {'nose', 'r_eye', 'l_eye', 'neck_base', 'spine', 'tail_base'}
