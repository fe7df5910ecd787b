"""Skeleton description tables for the cheetah kinematic tree.

The reference hard-codes its forward kinematics as straight-line numpy/sympy code
(`src/lib/misc.py:144-326`, marker lists `:8-49`, pose-parameter lists `:63-92`).
Here the same tree is expressed as *data*: a list of joints (rotation frames) and a
list of nodes (points). The HIP FK kernel (`csrc/fk.hip`) evaluates these tables, so
every mode the reference supports (`default`, `head`, `upper_body`,
`head_stabilize`) plus the 20-keypoint body used by the benchmarks
(`default_nolure`: `default` without `lure` and without `x_l, y_l, z_l`) is one table
and one kernel.

Conventions (restated from `src/lib/misc.py:381-420`): `rot_x/y/z` are passive
rotations; a joint's inertial->segment rotation is RI_j = R_a(t_a) @ R_b(t_b) @ ... @
RI_parent, and points are built as p = p_base + RI_j^T @ offset.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# --------------------------------------------------------------------------------------
# Marker lists / pose parameters (same names and order as src/lib/misc.py:8-92)
# --------------------------------------------------------------------------------------

_MARKERS = {
    'default': [
        'nose', 'r_eye', 'l_eye', 'neck_base',
        'spine', 'tail_base', 'tail1', 'tail2',
        'r_shoulder', 'r_front_knee', 'r_front_ankle',
        'l_shoulder', 'l_front_knee', 'l_front_ankle',
        'r_hip', 'r_back_knee', 'r_back_ankle',
        'l_hip', 'l_back_knee', 'l_back_ankle',
        'lure',
    ],
    'head': ['nose', 'r_eye', 'l_eye'],
    'upper_body': ['nose', 'r_eye', 'l_eye', 'neck_base', 'spine', 'r_shoulder', 'l_shoulder'],
    'head_stabilize': ['nose', 'r_eye', 'l_eye', 'neck_base', 'spine'],
    'all': [
        'nose', 'r_eye', 'l_eye', 'neck_base',
        'spine', 'tail_base', 'tail1', 'tail2',
        'r_shoulder', 'r_front_knee', 'r_front_ankle', 'r_front_paw',
        'l_shoulder', 'l_front_knee', 'l_front_ankle', 'l_front_paw',
        'r_hip', 'r_back_knee', 'r_back_ankle', 'r_back_paw',
        'l_hip', 'l_back_knee', 'l_back_ankle', 'l_back_paw',
        'lure',
    ],
}
_MARKERS['default_nolure'] = _MARKERS['default'][:20]

_POSE = {
    'default': [
        'x_0', 'y_0', 'z_0', 'phi_0', 'theta_0', 'psi_0',
        'l_1', 'phi_1', 'theta_1', 'psi_1', 'theta_2',
        'phi_3', 'theta_3', 'psi_3', 'theta_4', 'psi_4', 'theta_5', 'psi_5',
        'theta_6', 'theta_7', 'theta_8', 'theta_9',
        'theta_10', 'theta_11', 'theta_12', 'theta_13',
        'x_l', 'y_l', 'z_l',
    ],
    'head': ['x_0', 'y_0', 'z_0', 'phi_0', 'theta_0', 'psi_0'],
}
_POSE['upper_body'] = _POSE['default'][:11]
_POSE['head_stabilize'] = _POSE['default'][:11]
_POSE['default_nolure'] = _POSE['default'][:26]

FK_MODES = ('default', 'default_nolure', 'head', 'upper_body', 'head_stabilize')


def get_markers(mode: str = 'default', directions: bool = False) -> List[str]:
    """Marker names, `src/lib/misc.py:8-49`."""
    s = list(_MARKERS[mode])
    if directions:
        s += ['coe', 'gaze_target']
    return s


def get_skeleton() -> List[List[str]]:
    """Bone list, `src/lib/misc.py:52-60`."""
    return [
        ['nose', 'l_eye'], ['nose', 'r_eye'], ['nose', 'neck_base'], ['l_eye', 'neck_base'],
        ['r_eye', 'neck_base'], ['neck_base', 'spine'], ['spine', 'tail_base'],
        ['tail_base', 'tail1'], ['tail1', 'tail2'],
        ['neck_base', 'r_shoulder'], ['r_shoulder', 'r_front_knee'], ['r_front_knee', 'r_front_ankle'],
        ['neck_base', 'l_shoulder'], ['l_shoulder', 'l_front_knee'], ['l_front_knee', 'l_front_ankle'],
        ['tail_base', 'r_hip'], ['r_hip', 'r_back_knee'], ['r_back_knee', 'r_back_ankle'],
        ['tail_base', 'l_hip'], ['l_hip', 'l_back_knee'], ['l_back_knee', 'l_back_ankle'],
    ]


def get_pose_params(mode: str = 'default') -> Dict[str, int]:
    """Pose-parameter index, `src/lib/misc.py:63-92`."""
    states = _POSE[mode]
    return dict(zip(states, range(len(states))))


# --------------------------------------------------------------------------------------
# Tree tables
# --------------------------------------------------------------------------------------

AXIS = {'x': 0, 'y': 1, 'z': 2}

# Param kinds in the device table.
PK_TRANS, PK_ROT, PK_LEN, PK_WORLD = 0, 1, 2, 3
# Node base codes.
BASE_HEAD = -1    # p = p_head (x_0, y_0, z_0 [+ shutter shift])
BASE_WORLD = -2   # p = (x_l, y_l, z_l) (lure)


@dataclass
class Joint:
    name: str
    parent: int                        # -1 = inertial
    seq: List[Tuple[str, str]]         # [(axis, param)] in RI_local = R_a @ R_b @ ... order
    origin: str                        # node the rotation pivots about


@dataclass
class Node:
    name: str
    base: str                          # node name, or 'HEAD' / 'WORLD'
    frame: int                         # joint frame of the offset (-1 for HEAD / WORLD)
    offset: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    offset_param: Optional[str] = None  # x-offset taken from a pose parameter (neck length l_1)


_HEAD_OFFS_A = dict(l_eye=(0.0, 0.03, 0.0), r_eye=(0.0, -0.03, 0.0), nose=(0.055, 0.0, -0.055))
_E = 0.038852231676497324
_N = 0.0571868749393016
_HEAD_OFFS_B = dict(l_eye=(0.0, _E, 0.0), r_eye=(0.0, -_E, 0.0), nose=(_N, 0.0, -_N))

_JOINTS_FULL = [
    Joint('head', -1, [('z', 'psi_0'), ('x', 'phi_0'), ('y', 'theta_0')], 'head'),
    Joint('neck', 0, [('z', 'psi_1'), ('x', 'phi_1'), ('y', 'theta_1')], 'head'),
    Joint('front_torso', 1, [('y', 'theta_2')], 'neck_base'),
    Joint('back_torso', 2, [('z', 'psi_3'), ('x', 'phi_3'), ('y', 'theta_3')], 'spine'),
    Joint('tail_base', 3, [('z', 'psi_4'), ('y', 'theta_4')], 'tail_base'),
    Joint('tail_mid', 4, [('z', 'psi_5'), ('y', 'theta_5')], 'tail1'),
    Joint('l_shoulder', 2, [('y', 'theta_6')], 'l_shoulder'),
    Joint('l_front_knee', 6, [('y', 'theta_7')], 'l_front_knee'),
    Joint('r_shoulder', 2, [('y', 'theta_8')], 'r_shoulder'),
    Joint('r_front_knee', 8, [('y', 'theta_9')], 'r_front_knee'),
    Joint('l_hip', 3, [('y', 'theta_10')], 'l_hip'),
    Joint('l_back_knee', 10, [('y', 'theta_11')], 'l_back_knee'),
    Joint('r_hip', 3, [('y', 'theta_12')], 'r_hip'),
    Joint('r_back_knee', 12, [('y', 'theta_13')], 'r_back_knee'),
]


def _head_nodes(offs) -> List[Node]:
    return [Node('head', 'HEAD', -1),
            Node('l_eye', 'head', 0, offs['l_eye']),
            Node('r_eye', 'head', 0, offs['r_eye']),
            Node('nose', 'head', 0, offs['nose'])]


def _body_nodes() -> List[Node]:
    return [
        Node('neck_base', 'head', 1, (0.0, 0.0, 0.0), 'l_1'),
        Node('spine', 'neck_base', 2, (-0.37, 0.0, 0.0)),
        Node('tail_base', 'spine', 3, (-0.37, 0.0, 0.0)),
        Node('tail1', 'tail_base', 4, (-0.28, 0.0, 0.0)),
        Node('tail2', 'tail1', 5, (-0.36, 0.0, 0.0)),
        Node('l_shoulder', 'neck_base', 2, (-0.04, 0.08, -0.10)),
        Node('l_front_knee', 'l_shoulder', 6, (0.0, 0.0, -0.24)),
        Node('l_front_ankle', 'l_front_knee', 7, (0.0, 0.0, -0.28)),
        Node('r_shoulder', 'neck_base', 2, (-0.04, -0.08, -0.10)),
        Node('r_front_knee', 'r_shoulder', 8, (0.0, 0.0, -0.24)),
        Node('r_front_ankle', 'r_front_knee', 9, (0.0, 0.0, -0.28)),
        Node('l_hip', 'tail_base', 3, (0.12, 0.08, -0.06)),
        Node('l_back_knee', 'l_hip', 10, (0.0, 0.0, -0.32)),
        Node('l_back_ankle', 'l_back_knee', 11, (0.0, 0.0, -0.25)),
        Node('r_hip', 'tail_base', 3, (0.12, -0.08, -0.06)),
        Node('r_back_knee', 'r_hip', 12, (0.0, 0.0, -0.32)),
        Node('r_back_ankle', 'r_back_knee', 13, (0.0, 0.0, -0.25)),
    ]


def _tree(mode: str) -> Tuple[List[Joint], List[Node]]:
    if mode in ('default', 'default_nolure'):
        nodes = _head_nodes(_HEAD_OFFS_A) + _body_nodes()
        if mode == 'default':
            nodes.append(Node('lure', 'WORLD', -1))
        return list(_JOINTS_FULL), nodes
    if mode == 'head':
        return list(_JOINTS_FULL[:1]), _head_nodes(_HEAD_OFFS_B)
    if mode in ('upper_body', 'head_stabilize'):
        b = _body_nodes()
        keep = ['neck_base', 'spine'] + (['l_shoulder', 'r_shoulder'] if mode == 'upper_body' else [])
        return list(_JOINTS_FULL[:3]), _head_nodes(_HEAD_OFFS_B) + [n for n in b if n.name in keep]
    raise ValueError(f'unknown mode {mode!r}')


@dataclass
class SkeletonTable:
    """Flat int/float tables consumed by the HIP FK kernel (see include/acinoset_hip.h)."""
    mode: str
    P: int
    L: int
    n_joints: int
    n_nodes: int
    ints: np.ndarray      # int32 blob
    reals: np.ndarray     # float64 blob
    markers: List[str] = field(default_factory=list)
    params: List[str] = field(default_factory=list)


# int blob layout (all int32), see acs_skeleton in include/acinoset_hip.h:
#   [0] n_joints  [1] n_nodes  [2] P  [3] L  [4] head_node
#   joints  : n_joints * 8  -> parent, nrot, ax0, ax1, ax2, p0, p1, p2
#   joint_origin : n_joints
#   nodes   : n_nodes * 4   -> base_node (-1 head-root/-2 world), frame, offset_param, is_world
#   out_nodes : L
#   params  : P * 4         -> kind, a, b, c   (TRANS: axis; ROT: joint, seq idx; LEN: node; WORLD: axis)
#   deriv   : n_nodes * P   -> 1 if node depends on param
# real blob: nodes offsets n_nodes * 3
INT_HDR = 8


def build_table(mode: str) -> SkeletonTable:
    joints, nodes = _tree(mode)
    params = _POSE[mode]
    markers = _MARKERS[mode]
    pidx = {p: i for i, p in enumerate(params)}
    nidx = {n.name: i for i, n in enumerate(nodes)}
    P, L = len(params), len(markers)
    J, K = len(joints), len(nodes)

    # ancestors-or-self of each joint frame
    anc = []
    for j in range(J):
        s, k = set(), j
        while k >= 0:
            s.add(k)
            k = joints[k].parent
        anc.append(s)
    # frames and base-chain nodes used by each node
    frames_of, chain_of = [], []
    for k, n in enumerate(nodes):
        fr, ch = set(), {k}
        if n.frame >= 0:
            fr.add(n.frame)
        if n.base not in ('HEAD', 'WORLD'):
            b = nidx[n.base]
            fr |= frames_of[b]
            ch |= chain_of[b]
        frames_of.append(fr)
        chain_of.append(ch)

    deriv = np.zeros((K, P), np.int32)
    pk = np.zeros((P, 4), np.int32)
    for p, name in enumerate(params):
        if name in ('x_0', 'y_0', 'z_0'):
            pk[p] = (PK_TRANS, 'xyz'.index(name[0]), 0, 0)
            for k, n in enumerate(nodes):
                deriv[k, p] = 0 if n.base == 'WORLD' else 1
        elif name in ('x_l', 'y_l', 'z_l'):
            pk[p] = (PK_WORLD, 'xyz'.index(name[0]), 0, 0)
            for k, n in enumerate(nodes):
                deriv[k, p] = 1 if n.base == 'WORLD' else 0
        elif name == 'l_1':
            owner = [k for k, n in enumerate(nodes) if n.offset_param == 'l_1']
            assert len(owner) == 1
            pk[p] = (PK_LEN, owner[0], 0, 0)
            for k in range(K):
                deriv[k, p] = 1 if owner[0] in chain_of[k] else 0
        else:
            hit = [(j, r) for j, jt in enumerate(joints) for r, (_, pn) in enumerate(jt.seq) if pn == name]
            assert len(hit) == 1, name
            j, r = hit[0]
            pk[p] = (PK_ROT, j, r, 0)
            for k in range(K):
                deriv[k, p] = 1 if any(j in anc[f] for f in frames_of[k]) else 0

    ints: List[int] = [J, K, P, L, nidx['head'], 0, 0, 0]
    for jt in joints:
        axes = [AXIS[a] for a, _ in jt.seq] + [0] * (3 - len(jt.seq))
        ps = [pidx[pn] for _, pn in jt.seq] + [0] * (3 - len(jt.seq))
        ints += [jt.parent, len(jt.seq)] + axes + ps
    ints += [nidx[jt.origin] for jt in joints]
    for n in nodes:
        if n.base == 'HEAD':
            base = -1
        elif n.base == 'WORLD':
            base = -2
        else:
            base = nidx[n.base]
        ints += [base, n.frame, pidx[n.offset_param] if n.offset_param else -1, 1 if n.base == 'WORLD' else 0]
    ints += [nidx[m] for m in markers]
    ints += pk.ravel().tolist()
    ints += deriv.ravel().tolist()
    reals = np.array([c for n in nodes for c in n.offset], np.float64)
    return SkeletonTable(mode, P, L, J, K, np.asarray(ints, np.int32), reals, list(markers), list(params))


def fk_numpy(mode: str, x: np.ndarray, shift: Optional[np.ndarray] = None,
             directions: bool = False) -> np.ndarray:
    """Table-driven FK on the host, used ONLY by the synthetic data generator
    (`acinoset_amd.synth`) to make ground truth; solves never call it.

    x: (N, P); shift: (N, 3) added to the head position (shutter-delay shift,
    `src/lib/misc.py:190-193`). Returns (N, L[+2], 3).
    """
    joints, nodes = _tree(mode)
    params = _POSE[mode]
    pidx = {p: i for i, p in enumerate(params)}
    nidx = {n.name: i for i, n in enumerate(nodes)}
    x = np.atleast_2d(np.asarray(x, np.float64))
    N = x.shape[0]

    def act(axis, a):  # active rotation = rot_<axis>(a).T
        c, s = np.cos(a), np.sin(a)
        R = np.zeros((N, 3, 3))
        i, j = [(1, 2), (2, 0), (0, 1)][AXIS[axis]]
        k = AXIS[axis]
        R[:, k, k] = 1.0
        R[:, i, i] = c
        R[:, j, j] = c
        R[:, i, j] = -s
        R[:, j, i] = s
        return R

    M = []
    for jt in joints:
        G = np.broadcast_to(np.eye(3), (N, 3, 3)).copy()
        for axis, pn in jt.seq:          # G = A_last ... A_0 (A = R^T)
            G = act(axis, x[:, pidx[pn]]) @ G
        M.append(G if jt.parent < 0 else M[jt.parent] @ G)
    pos = np.zeros((N, len(nodes), 3))
    for k, n in enumerate(nodes):
        if n.base == 'HEAD':
            pos[:, k] = x[:, [pidx['x_0'], pidx['y_0'], pidx['z_0']]]
            if shift is not None:
                pos[:, k] += shift
        elif n.base == 'WORLD':
            pos[:, k] = x[:, [pidx['x_l'], pidx['y_l'], pidx['z_l']]]
        else:
            off = np.broadcast_to(np.asarray(n.offset), (N, 3)).copy()
            if n.offset_param:
                off[:, 0] = x[:, pidx[n.offset_param]]
            pos[:, k] = pos[:, nidx[n.base]] + np.einsum('nij,nj->ni', M[n.frame], off)
    out = pos[:, [nidx[m] for m in _MARKERS[mode]]]
    if directions:
        h = pos[:, nidx['head']]
        gaze = h + np.einsum('nij,j->ni', M[0], np.array([3.0, 0.0, 0.0]))
        out = np.concatenate([out, h[:, None], gaze[:, None]], axis=1)
    return out
