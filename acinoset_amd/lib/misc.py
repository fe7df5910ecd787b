"""Mirror of src/lib/misc.py: marker/pose tables, forward kinematics, loss.

`get_3d_marker_coords` / `get_all_marker_coords_from_states` evaluate the kinematic tree
on the GPU (acs_fk); `redescending_loss` runs on the GPU (acs_redescending_loss). The
symbolic (sympy) branch of the reference existed only to build the Pyomo model, which
this core replaces; passing sympy symbols raises TypeError.
"""
from typing import Dict, List

import numpy as np

from .. import _native
from ..kinematics import build_table, get_markers, get_pose_params, get_skeleton  # noqa: F401

_TABLES = {}


def _table(mode):
    if mode not in _TABLES:
        _TABLES[mode] = build_table(mode)
    return _TABLES[mode]


def _numeric(x):
    a = np.asarray(x)
    if a.dtype == object:
        raise TypeError('symbolic states are not supported: the Pyomo/sympy model is replaced by acs_fte_solve')
    return a.astype(np.float64)


def get_3d_marker_coords(states: Dict, tau: float = 0.0, directions: bool = False, mode: str = 'default',
                         intermode: str = 'pos'):
    """`src/lib/misc.py:144` for one state vector -> (L[+2], 3)."""
    x = _numeric(states['x']).reshape(1, -1)
    t = _table(mode)
    im = {'pos': 0, 'vel': 1, 'acc': 2}.get(intermode, 0)
    dx = states.get('dx')
    ddx = states.get('ddx')
    dxa = np.zeros_like(x) if dx is None or im < 1 else _numeric(dx).reshape(1, -1)
    ddxa = np.zeros_like(x) if ddx is None or im < 2 else _numeric(ddx).reshape(1, -1)
    out = _native.default_context().fk(t, x, dxa, ddxa, np.array([float(tau)]), intermode=im if im else 0,
                                       directions=directions)
    return out[0]


def get_all_marker_coords_from_states(states, n_cam: int, directions: bool = False, mode: str = 'default',
                                      intermode: str = 'pos') -> List:
    """`src/lib/misc.py:126-141`: per camera, (N, L[+2], 3) positions (shutter-delay shift per camera)."""
    t = _table(mode)
    x = _numeric(states['x'])
    sd = states.get('shutter_delay')
    ctx = _native.default_context()
    out = []
    for i in range(n_cam):
        if sd is not None:
            im = {'pos': 0, 'vel': 1, 'acc': 2}.get(intermode, 0)
            dx = _numeric(states['dx']) if im >= 1 else np.zeros_like(x)
            ddx = _numeric(states['ddx']) if im >= 2 else np.zeros_like(x)
            out.append(ctx.fk(t, x, dx, ddx, _numeric(sd[i]), intermode=im, directions=directions))
        else:
            out.append(ctx.fk(t, x, directions=directions))
    return out


def redescending_loss(err, a, b, c):
    """`src/lib/misc.py:329-343` (elementwise, GPU)."""
    e = np.asarray(err, np.float64)
    v = _native.default_context().redescending_loss(e.ravel(), float(a), float(b), float(c))
    return v.reshape(e.shape) if e.shape else float(v[0])


def rot_x(x):
    c, s = np.cos(x), np.sin(x)
    return np.array([[1, 0, 0], [0, c, s], [0, -s, c]])


def rot_y(y):
    c, s = np.cos(y), np.sin(y)
    return np.array([[c, 0, -s], [0, 1, 0], [s, 0, c]])


def rot_z(z):
    c, s = np.cos(z), np.sin(z)
    return np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])


def global_positions(R_arr, t_arr):
    """Camera centres -R^T t (`src/lib/misc.py:346-357`)."""
    R = np.asarray(R_arr, np.float64).reshape(-1, 3, 3)
    t = np.asarray(t_arr, np.float64).reshape(-1, 3, 1)
    return np.array([-r.T @ tt for r, tt in zip(R, t)], dtype=np.float32)


class Logger:
    """stdout tee (`src/lib/misc.py:424-438`)."""

    def __init__(self, out_fpath):
        import sys
        self.terminal = sys.stdout
        self.logfile = open(out_fpath, 'w', buffering=1)

    def write(self, message):
        self.terminal.write(message)
        self.logfile.write(message)

    def flush(self):
        pass
