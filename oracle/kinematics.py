"""Oracle: cheetah forward kinematics and the redescending loss.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* `marker_positions` restates `get_3d_marker_coords` (`src/lib/misc.py:144-326`) for
  the numeric case, vectorised over frames and written so that it also runs on
  complex inputs (complex-step differentiation gives the oracle an exact FK
  Jacobian). Pinned by tests/golden/fk.npz (reference outputs).
* `redescending_loss` restates `src/lib/misc.py:329-343`; pinned by
  tests/golden/loss.npz. `loss_d1`/`loss_d2` are its analytic derivatives in |e|.
"""
import numpy as np

POSE = {
    'default': ['x_0', 'y_0', 'z_0', 'phi_0', 'theta_0', 'psi_0', 'l_1', 'phi_1', 'theta_1', 'psi_1', 'theta_2',
                'phi_3', 'theta_3', 'psi_3', 'theta_4', 'psi_4', 'theta_5', 'psi_5', 'theta_6', 'theta_7',
                'theta_8', 'theta_9', 'theta_10', 'theta_11', 'theta_12', 'theta_13', 'x_l', 'y_l', 'z_l'],
    'head': ['x_0', 'y_0', 'z_0', 'phi_0', 'theta_0', 'psi_0'],
}
POSE['upper_body'] = POSE['default'][:11]
POSE['head_stabilize'] = POSE['default'][:11]
POSE['default_nolure'] = POSE['default'][:26]


def _cs(a, f32):
    """cos, sin; with f32 evaluated in float32 on float32-rounded angles (the numerics of the
    reference EKF, whose predicted states are float32: src/core/ekf.py:79, misc.py:381-420)."""
    if f32:
        a32 = np.asarray(a).astype(np.float32)
        return np.cos(a32).astype(np.float64), np.sin(a32).astype(np.float64)
    return np.cos(a), np.sin(a)


def _rx0(a, f32=False):
    c, s = _cs(a, f32)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([o, z, z], -1), np.stack([z, c, s], -1), np.stack([z, -s, c], -1)], -2)


def _ry0(a, f32=False):
    c, s = _cs(a, f32)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([c, z, -s], -1), np.stack([z, o, z], -1), np.stack([s, z, c], -1)], -2)


def _rz0(a, f32=False):
    c, s = _cs(a, f32)
    o, z = np.ones_like(a), np.zeros_like(a)
    return np.stack([np.stack([c, s, z], -1), np.stack([-s, c, z], -1), np.stack([z, z, o], -1)], -2)


def _app(R, v):
    """R^T @ v for stacked R (n,3,3) and constant or stacked v."""
    v = np.asarray(v)
    if v.ndim == 1:
        return np.einsum('nji,j->ni', R, v)
    return np.einsum('nji,nj->ni', R, v)


def marker_positions(mode, x, shift=None, directions=False, f32_trig=False):
    """x (n, P) real or complex -> (n, L[+2], 3). `shift` (n,3) is added to p_head.
    `f32_trig`: rotation cos/sin in float32 (see _cs)."""
    x = np.atleast_2d(x)
    _rx = lambda a: _rx0(a, f32_trig)  # noqa: E731
    _ry = lambda a: _ry0(a, f32_trig)  # noqa: E731
    _rz = lambda a: _rz0(a, f32_trig)  # noqa: E731
    idx = {k: i for i, k in enumerate(POSE[mode])}
    X = lambda k: x[:, idx[k]]  # noqa: E731
    n = x.shape[0]
    RI_0 = _rz(X('psi_0')) @ _rx(X('phi_0')) @ _ry(X('theta_0'))
    p_head = np.stack([X('x_0'), X('y_0'), X('z_0')], -1)
    if shift is not None:
        p_head = p_head + shift
    if mode in ('default', 'default_nolure'):
        eye, nose = 0.03, (0.055, 0.0, -0.055)
    else:
        e_, n_ = 0.038852231676497324, 0.0571868749393016
        eye, nose = e_, (n_, 0.0, -n_)
    p_l_eye = p_head + _app(RI_0, [0, eye, 0])
    p_r_eye = p_head + _app(RI_0, [0, -eye, 0])
    p_nose = p_head + _app(RI_0, list(nose))
    out = [p_nose, p_r_eye, p_l_eye]
    if mode != 'head':
        RI_1 = _rz(X('psi_1')) @ _rx(X('phi_1')) @ _ry(X('theta_1')) @ RI_0
        RI_2 = _ry(X('theta_2')) @ RI_1
        z = np.zeros(n, dtype=x.dtype)
        p_neck = p_head + _app(RI_1, np.stack([X('l_1'), z, z], -1))
        p_spine = p_neck + _app(RI_2, [-0.37, 0, 0])
        if mode == 'upper_body':
            out += [p_neck, p_spine, p_neck + _app(RI_2, [-0.04, -0.08, -0.10]),
                    p_neck + _app(RI_2, [-0.04, 0.08, -0.10])]
        elif mode == 'head_stabilize':
            out += [p_neck, p_spine]
        else:
            RI_3 = _rz(X('psi_3')) @ _rx(X('phi_3')) @ _ry(X('theta_3')) @ RI_2
            RI_4 = _rz(X('psi_4')) @ _ry(X('theta_4')) @ RI_3
            RI_5 = _rz(X('psi_5')) @ _ry(X('theta_5')) @ RI_4
            RI_6 = _ry(X('theta_6')) @ RI_2
            RI_7 = _ry(X('theta_7')) @ RI_6
            RI_8 = _ry(X('theta_8')) @ RI_2
            RI_9 = _ry(X('theta_9')) @ RI_8
            RI_10 = _ry(X('theta_10')) @ RI_3
            RI_11 = _ry(X('theta_11')) @ RI_10
            RI_12 = _ry(X('theta_12')) @ RI_3
            RI_13 = _ry(X('theta_13')) @ RI_12
            p_tb = p_spine + _app(RI_3, [-0.37, 0, 0])
            p_t1 = p_tb + _app(RI_4, [-0.28, 0, 0])
            p_t2 = p_t1 + _app(RI_5, [-0.36, 0, 0])
            p_ls = p_neck + _app(RI_2, [-0.04, 0.08, -0.10])
            p_lfk = p_ls + _app(RI_6, [0, 0, -0.24])
            p_lfa = p_lfk + _app(RI_7, [0, 0, -0.28])
            p_rs = p_neck + _app(RI_2, [-0.04, -0.08, -0.10])
            p_rfk = p_rs + _app(RI_8, [0, 0, -0.24])
            p_rfa = p_rfk + _app(RI_9, [0, 0, -0.28])
            p_lh = p_tb + _app(RI_3, [0.12, 0.08, -0.06])
            p_lbk = p_lh + _app(RI_10, [0, 0, -0.32])
            p_lba = p_lbk + _app(RI_11, [0, 0, -0.25])
            p_rh = p_tb + _app(RI_3, [0.12, -0.08, -0.06])
            p_rbk = p_rh + _app(RI_12, [0, 0, -0.32])
            p_rba = p_rbk + _app(RI_13, [0, 0, -0.25])
            out += [p_neck, p_spine, p_tb, p_t1, p_t2, p_rs, p_rfk, p_rfa, p_ls, p_lfk, p_lfa,
                    p_rh, p_rbk, p_rba, p_lh, p_lbk, p_lba]
            if mode == 'default':
                out.append(np.stack([X('x_l'), X('y_l'), X('z_l')], -1))
    if directions:
        out += [p_head, p_head + _app(RI_0, [3, 0, 0])]
    return np.stack(out, 1)


def marker_jacobian(mode, x):
    """Exact d positions / d x by complex step: (n, L, 3, P)."""
    x = np.atleast_2d(np.asarray(x, np.float64))
    n, P = x.shape
    h = 1e-30
    cols = []
    for p in range(P):
        xc = x.astype(np.complex128)
        xc[:, p] += 1j * h
        cols.append(marker_positions(mode, xc).imag / h)
    return np.stack(cols, -1)


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def redescending_loss(err, a=3.0, b=10.0, c=20.0):
    e = np.abs(err)
    sa, sb, sc = _sig(e - a), _sig(e - b), _sig(e - c)
    return ((1 - sa) / 2 * e ** 2 + (sa - sb) * (a * e - a * a / 2)
            + (sb - sc) * (a * b - a * a / 2 + (a * (c - b) / 2) * (1 - ((c - e) / (c - b)) ** 2))
            + sc * (a * b - a * a / 2 + a * (c - b) / 2))


def loss_derivs(err, a=3.0, b=10.0, c=20.0):
    """(rho'(err), rho''(err)) — analytic, in err (sign folded into rho')."""
    e = np.abs(err)
    sa, sb, sc = _sig(e - a), _sig(e - b), _sig(e - c)
    da, db, dc = sa * (1 - sa), sb * (1 - sb), sc * (1 - sc)
    dda, ddb, ddc = da * (1 - 2 * sa), db * (1 - 2 * sb), dc * (1 - 2 * sc)
    lin = a * e - a * a / 2
    K3 = a * b - a * a / 2
    w = (c - e) / (c - b)
    q = K3 + (a * (c - b) / 2) * (1 - w * w)
    q1 = a * (c - e) / (c - b)
    q2 = -a / (c - b)
    K4 = K3 + a * (c - b) / 2
    d1 = (-0.5 * da * e * e + (1 - sa) * e + (da - db) * lin + (sa - sb) * a + (db - dc) * q + (sb - sc) * q1
          + dc * K4)
    d2 = (-0.5 * dda * e * e - 2 * da * e + (1 - sa) + (dda - ddb) * lin + 2 * (da - db) * a + (ddb - ddc) * q
          + 2 * (db - dc) * q1 + (sb - sc) * q2 + ddc * K4)
    return d1 * np.sign(err), d2
