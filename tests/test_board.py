"""Calibration-board bundle adjustment front end (src/lib/sba.py:37-137, :209-282) against
the reference's own run (tests/golden/board.npz, made by tests/golden/make_golden.py
board: the reference's prepare_* functions and _sba_board_points with the numpy cv2
shim). CPU tests inject the oracle triangulation through the triangulate_func seam; the
GPU test runs the drop-in end to end (GPU triangulation + points/extrinsics SBA)."""
import json
import os

import numpy as np
import pytest

from acinoset_amd.lib import sba as lsba
from acinoset_amd.lib import utils as lutils
from oracle import fisheye as ofish
from oracle import sba_ext as oext

G = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'board.npz'))
C = len(G['K'])


def _tri(a, b, ka, da, ra, ta, kb, db, rb, tb):
    return ofish.triangulate_pair(np.asarray(a, np.float64).reshape(-1, 2), np.asarray(b, np.float64).reshape(-1, 2),
                                  ka, np.ravel(da), ra, np.ravel(ta), kb, np.ravel(db), rb, np.ravel(tb))


def _files(tmp_path):
    pfs = []
    for c in range(C):
        p = tmp_path / f'points_cam{c}.json'
        p.write_text(str(G[f'points_cam{c}']))
        pfs.append(str(p))
    mf = tmp_path / 'manual_points.json'
    mf.write_text(str(G['manual_points_json']))
    scene = tmp_path / 'scene.json'
    lutils.save_scene(str(scene), G['K'], G['D'], G['R0'], G['t0'], tuple(int(v) for v in G['res']))
    return str(scene), pfs, str(mf)


def _board_inputs(pfs):
    img, fns = [], []
    for pf in pfs:
        p, fn, shape, *_ = lutils.load_points(pf)
        img.append(p)
        fns.append(fn)
    return img, fns, shape


def _reorder(p2, p3, pi, ci, ppi):
    """Our image-name order (sorted) -> the reference's (a set's iteration order)."""
    order = [str(s) for s in G['board_fname_order']]
    ours = sorted(order)
    rows, pts = [], []
    for fn in order:
        b = ours.index(fn)
        pts.append(p3[b * ppi:(b + 1) * ppi])
        rows.append(np.flatnonzero((pi >= b * ppi) & (pi < (b + 1) * ppi)))
    rows = np.concatenate(rows)
    blk = {ours.index(fn): k for k, fn in enumerate(order)}
    pi_new = np.array([blk[i // ppi] * ppi + i % ppi for i in pi[rows]])
    return p2[rows], np.concatenate(pts), pi_new, ci[rows], rows


def test_load_points_schema(tmp_path):
    _, pfs, mf = _files(tmp_path)
    p, fn, shape, sq, res = lutils.load_points(pfs[0])
    assert p.dtype == np.float32 and p.shape[1:] == (int(np.prod(G['board_shape'])), 1, 2)
    assert shape == tuple(G['board_shape']) and sq == float(G['square'])
    m, mfn, _ = lutils.load_manual_points(mf, verbose=False)
    np.testing.assert_array_equal(np.isnan(m), np.isnan(G['manual']))
    assert mfn[0] == 'img00000.jpg'
    lutils.save_points(str(tmp_path / 'rt.json'), p, fn, shape, sq, res)
    p2, fn2, *_ = lutils.load_points(str(tmp_path / 'rt.json'))
    np.testing.assert_array_equal(p2, p)
    assert fn2 == fn


def test_board_data_prep_matches_reference(tmp_path):
    _, pfs, _ = _files(tmp_path)
    img, fns, shape = _board_inputs(pfs)
    p2, p3, pi, ci = lsba.prepare_calib_board_data_for_bundle_adjustment(img, fns, shape, G['K'], G['D'], G['R0'],
                                                                         G['t0'], _tri)
    assert p2.dtype == np.float32 and p3.dtype == np.float32
    p2, p3, pi, ci, _ = _reorder(p2, p3, pi, ci, int(np.prod(shape)))
    np.testing.assert_array_equal(p2, G['board_points_2d'])
    np.testing.assert_array_equal(pi, G['board_point_indices'])
    np.testing.assert_array_equal(ci, G['board_camera_indices'])
    # float32 of the same triangulation (oracle restatement vs the reference through the shim)
    np.testing.assert_allclose(p3, G['board_points_3d'], atol=2e-6)


def test_manual_data_prep_matches_reference():
    m2, m3, mi, mc = lsba.prepare_manual_points_for_bundle_adjustment(G['manual'], G['K'], G['D'], G['R0'], G['t0'],
                                                                      _tri)
    np.testing.assert_array_equal(m2, G['manual_points_2d'])
    np.testing.assert_array_equal(mi, G['manual_point_indices'])
    np.testing.assert_array_equal(mc, G['manual_camera_indices'])
    np.testing.assert_allclose(m3, G['manual_points_3d'], atol=2e-6)


def _ref_problem():
    p2 = np.concatenate([G['board_points_2d'], G['manual_points_2d']]).astype(np.float64)
    p3 = np.concatenate([G['board_points_3d'], G['manual_points_3d']]).astype(np.float64)
    bi = G['board_point_indices']
    pi = np.concatenate([bi, G['manual_point_indices'] + bi.max()])   # src/lib/sba.py:249
    ci = np.concatenate([G['board_camera_indices'], G['manual_camera_indices']])
    return p2, p3, pi, ci


def test_reference_objective_on_golden_problem():
    """The golden residuals are the reference's, on the problem the prep produced."""
    p2, p3, pi, ci = _ref_problem()
    r = oext.residuals(p3, G['R0'], G['t0'].reshape(-1, 3), G['K'], G['D'].reshape(-1, 4), p2, pi, ci)
    np.testing.assert_allclose(r.ravel(), G['resid_before'], atol=1e-6)


@pytest.mark.gpu
def test_sba_board_points_dropin(tmp_path):
    from acinoset_amd.lib import app
    scene, pfs, mf = _files(tmp_path)
    out = str(tmp_path / 'scene_sba.json')
    res = app.sba_board_points_fisheye(scene, pfs, out, manual_points_fpath=mf)
    # observation order: board rows by image name (ours sorted, the reference's a set's
    # order), then the manual rows in the same order
    img, fns, shape = _board_inputs(pfs)
    p2, p3, pi, ci = lsba.prepare_calib_board_data_for_bundle_adjustment(img, fns, shape, G['K'], G['D'], G['R0'],
                                                                         G['t0'])
    np.testing.assert_allclose(_reorder(p2, p3, pi, ci, int(np.prod(shape)))[1], G['board_points_3d'], atol=2e-6)
    rows = np.concatenate([_reorder(p2, p3, pi, ci, int(np.prod(shape)))[4], len(p2) + np.arange(len(G['manual_points_2d']))])
    before = np.asarray(res['before']).reshape(-1, 2)[rows]
    # manual point 0 shares its index with the LAST board point (src/lib/sba.py:249), which
    # depends on the image-name order: its observations are compared on the cost only
    keep = np.concatenate([np.ones(len(G['board_points_2d']), bool), G['manual_point_indices'] != 0])
    np.testing.assert_allclose(before[keep], G['resid_before'].reshape(-1, 2)[keep], atol=5e-3)  # float32 init
    k, d, R, t, _ = lutils.load_scene(out, verbose=False)

    def cauchy(r):
        return 0.5 * np.sum(np.log1p(np.asarray(r) ** 2))   # f_scale = 1 (src/lib/sba.py:170)
    # same objective, at least as low as the reference's scipy TRF run reached
    assert cauchy(res['after']) <= cauchy(G['resid_after']) * (1 + 1e-6)
    with open(out) as f:
        assert len(json.load(f)['cameras']) == C
    for c in range(C):
        np.testing.assert_allclose(R[c] @ R[c].T, np.eye(3), atol=1e-10)
