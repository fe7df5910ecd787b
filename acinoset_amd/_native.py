"""ctypes binding of libacinoset_hip.so (the C ABI in include/acinoset_hip.h).

There is no CPU fallback: if the shared library is missing, or no gfx950 device is
visible, every call raises `NativeUnavailable` loudly.

`torch` is imported (if installed) BEFORE the library is loaded, so that the process
has a single HIP runtime: torch bundles its own libamdhip64.so.7 and the library's
NEEDED entry then binds to that already-loaded copy.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import numpy as np

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the product
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ACINOSET_HIP_LIB', os.path.join(_HERE, 'libacinoset_hip.so'))

ACS_DEVICE_PTRS = 1
ACS_CAM_STRIDE = 20
STATUS_NAMES = ('running', 'gtol', 'ftol', 'xtol', 'stalled', 'maxiter', 'noobs')
SD_MODES = {'const': 0, 'variable': 1}        # src/core/fte.py:35 shutter_delay_mode

# exported symbols (checked by tests against include/acinoset_hip.h)
SYMBOLS = (
    'acs_ctx_create', 'acs_ctx_destroy', 'acs_last_error', 'acs_ctx_set_stream', 'acs_ctx_sync',
    'acs_abi_version', 'acs_device_count', 'acs_sba_default_opts', 'acs_project_fisheye',
    'acs_sba_residuals', 'acs_sba_points', 'acs_sba_points_dense', 'acs_redescending_loss', 'acs_fk',
    'acs_fte_default_opts', 'acs_fte_solve', 'acs_fte_eval', 'acs_triangulate_pairs', 'acs_triangulate_dense',
    'acs_sba_ext_default_opts', 'acs_sba_extrinsics', 'acs_sba_points_dense_io',
    'acs_fte_dist_create', 'acs_fte_dist_init', 'acs_fte_dist_round', 'acs_fte_dist_poll',
    'acs_fte_dist_gather', 'acs_fte_dist_scatter', 'acs_fte_dist_result',
    'acs_fte_dist_destroy', 'acs_fte_dist_reset', 'acs_alloc_events', 'acs_ekf_singular_count',
    'acs_fte_debug_blocks',
    'acs_sba_ext_dist_create', 'acs_sba_ext_dist_init', 'acs_sba_ext_dist_round', 'acs_sba_ext_dist_poll',
    'acs_sba_ext_dist_result', 'acs_sba_ext_dist_destroy', 'acs_ekf_run',
    'acs_sba_ekf_pipeline',
)


class NativeUnavailable(RuntimeError):
    pass


class SbaOpts(C.Structure):
    _fields_ = [('max_iters', C.c_int32), ('reserved', C.c_int32), ('f_scale', C.c_double),
                ('ftol', C.c_double), ('xtol', C.c_double), ('gtol', C.c_double)]


class Report(C.Structure):
    _fields_ = [('n_problems', C.c_int64), ('status_counts', C.c_int64 * 7), ('iters_max', C.c_int64),
                ('iters_sum', C.c_int64), ('nfev_sum', C.c_int64), ('cost_before', C.c_double),
                ('cost_after', C.c_double)]

    def as_dict(self):
        return dict(n_problems=self.n_problems,
                    status_counts={STATUS_NAMES[i]: int(self.status_counts[i]) for i in range(7)},
                    iters_max=self.iters_max, iters_sum=self.iters_sum, nfev_sum=self.nfev_sum,
                    cost_before=self.cost_before, cost_after=self.cost_after)


class EkfInitSpec(C.Structure):
    """acs_ekf_init_spec: what the EKF's initial state is fitted on (src/core/ekf.py:121-157)."""
    _fields_ = [(k, C.c_int32) for k in ('nose', 'lure', 'x0', 'y0', 'psi0', 'xl', 'yl', 'from_sba')]


def ekf_numerics_mode(ref_numerics, jacobian):
    """The C ABI's EKF measurement-model mode: 1 = the reference's float32 numerics with the
    forward-difference H, 0 = the same H in float64, ACS_EKF_ANALYTIC_H (2) = the analytic H
    (float64 only)."""
    if jacobian == 'analytic':
        if ref_numerics:
            raise ValueError("jacobian='analytic' runs in float64: pass ref_numerics=False")
        return 2
    if jacobian != 'fd':
        raise ValueError(f"jacobian must be 'fd' or 'analytic', not {jacobian!r}")
    return int(bool(ref_numerics))


def ekf_init_spec(table, obs_markers, from_sba=False):
    """The pipeline's init descriptor for EKF skeleton `table` on observations whose marker
    order is `obs_markers`."""
    obs = list(obs_markers)
    pidx = {p: i for i, p in enumerate(table.params)}
    lure = obs.index('lure') if ('lure' in table.markers and 'lure' in obs) else -1
    return EkfInitSpec(obs.index('nose'), lure, pidx['x_0'], pidx['y_0'], pidx['psi_0'], pidx.get('x_l', -1),
                       pidx.get('y_l', -1), int(bool(from_sba)))


class FteOpts(C.Structure):
    _fields_ = [('max_iters', C.c_int32), ('window', C.c_int32), ('ftol', C.c_double), ('xtol', C.c_double),
                ('gtol', C.c_double), ('lambda0', C.c_double), ('redesc_a', C.c_double),
                ('redesc_b', C.c_double), ('redesc_c', C.c_double)]


class FteReport(C.Structure):
    _fields_ = [('status', C.c_int32), ('iters', C.c_int32), ('n_accepted', C.c_int32), ('n_bad_pivots', C.c_int32),
                ('cost_before', C.c_double), ('cost_after', C.c_double), ('cost_meas', C.c_double),
                ('cost_model', C.c_double), ('grad_max', C.c_double), ('lambda_final', C.c_double)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d['status_name'] = STATUS_NAMES[self.status] if 0 <= self.status < 7 else str(self.status)
        return d


class SbaExtOpts(C.Structure):
    _fields_ = [('max_iters', C.c_int32), ('reserved', C.c_int32), ('f_scale', C.c_double), ('ftol', C.c_double),
                ('xtol', C.c_double), ('gtol', C.c_double), ('lambda0', C.c_double)]


class SbaExtReport(C.Structure):
    _fields_ = [('status', C.c_int32), ('iters', C.c_int32), ('n_accepted', C.c_int32), ('n_bad_pivots', C.c_int32),
                ('cost_before', C.c_double), ('cost_after', C.c_double), ('grad_max', C.c_double),
                ('lambda_final', C.c_double)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d['status_name'] = STATUS_NAMES[self.status] if 0 <= self.status < 7 else str(self.status)
        return d


# must equal ACS_ABI_VERSION in include/acinoset_hip.h (checked when the library loads)
ABI_VERSION = 5
_lib = None
_lock = threading.Lock()
_P = C.c_void_p
_D = C.POINTER(C.c_double)


def _declare(lib):
    i32, i64, u32, dbl = C.c_int32, C.c_int64, C.c_uint32, C.c_double
    sig = {
        'acs_ctx_create': (C.c_int, [C.c_int, C.POINTER(_P)]),
        'acs_ctx_destroy': (C.c_int, [_P]),
        'acs_last_error': (C.c_char_p, [_P]),
        'acs_ctx_set_stream': (C.c_int, [_P, _P]),
        'acs_ctx_sync': (C.c_int, [_P]),
        'acs_abi_version': (C.c_int, []),
        'acs_device_count': (C.c_int, [C.POINTER(C.c_int)]),
        'acs_sba_default_opts': (None, [C.POINTER(SbaOpts)]),
        'acs_project_fisheye': (C.c_int, [_P, _P, i32, _P, _P, i64, i32, _P, u32]),
        'acs_sba_residuals': (C.c_int, [_P, _P, i32, _P, _P, _P, i64, _P, i64, _P, u32]),
        'acs_sba_points': (C.c_int, [_P, _P, i32, _P, _P, _P, i64, _P, i64, C.POINTER(SbaOpts), _P, _P,
                                     C.POINTER(Report), u32]),
        'acs_sba_points_dense': (C.c_int, [_P, _P, i32, _P, _P, i64, _P, C.POINTER(SbaOpts), C.POINTER(Report),
                                           u32]),
        'acs_sba_points_dense_io': (C.c_int, [_P, _P, i32, _P, _P, i64, _P, _P, C.POINTER(SbaOpts),
                                              C.POINTER(Report), u32]),
        'acs_redescending_loss': (C.c_int, [_P, _P, i64, dbl, dbl, dbl, _P, _P, u32]),
        'acs_fk': (C.c_int, [_P, _P, i64, _P, i64, _P, _P, _P, _P, i64, i32, i32, _P, _P, u32]),
        'acs_fte_default_opts': (None, [C.POINTER(FteOpts)]),
        'acs_fte_solve': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, dbl, _P, i32, i32, _P, _P,
                                    C.POINTER(FteOpts), C.POINTER(FteReport), u32]),
        'acs_fte_eval': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, dbl, _P, i32, i32, _P, _P,
                                   _P, _P, _P, u32]),
        'acs_fte_debug_blocks': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, dbl, _P, i32, i32, _P, _P,
                                           dbl, i32, _P, C.POINTER(i64), u32]),
        'acs_triangulate_pairs': (C.c_int, [_P, _P, i32, _P, _P, _P, _P, i64, _P, u32]),
        'acs_triangulate_dense': (C.c_int, [_P, _P, i32, _P, _P, i64, _P, _P, u32]),
        'acs_sba_ext_default_opts': (None, [C.POINTER(SbaExtOpts)]),
        'acs_fte_dist_create': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, dbl, _P, i32, i32, _P, _P,
                                          C.POINTER(FteOpts), i32, i32, C.POINTER(_P), C.POINTER(i64), u32]),
        'acs_fte_dist_init': (C.c_int, [_P, _P]),
        'acs_fte_dist_round': (C.c_int, [_P, _P, _P]),
        'acs_fte_dist_poll': (C.c_int, [_P, i64, C.POINTER(i32)]),
        'acs_fte_dist_gather': (C.c_int, [_P, _P]),
        'acs_fte_dist_scatter': (C.c_int, [_P, _P]),
        'acs_fte_dist_result': (C.c_int, [_P, _P, _P, C.POINTER(FteReport), u32]),
        'acs_fte_dist_destroy': (C.c_int, [_P]),
        'acs_fte_dist_reset': (C.c_int, [_P, _P, _P, u32]),
        'acs_alloc_events': (C.c_int64, []),
        'acs_ekf_singular_count': (C.c_int, [_P, C.POINTER(i32)]),
        'acs_sba_ext_dist_create': (C.c_int, [_P, _P, i32, _P, _P, _P, i64, _P, i64, C.POINTER(SbaExtOpts), i32, i32,
                                              C.POINTER(_P), C.POINTER(i64), u32]),
        'acs_sba_ext_dist_init': (C.c_int, [_P, _P]),
        'acs_sba_ext_dist_round': (C.c_int, [_P, _P, _P]),
        'acs_sba_ext_dist_poll': (C.c_int, [_P, C.c_int64, C.POINTER(i32)]),
        'acs_sba_ext_dist_result': (C.c_int, [_P, _P, _P, C.POINTER(SbaExtReport), u32]),
        'acs_sba_ext_dist_destroy': (C.c_int, [_P]),
        'acs_ekf_run': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, dbl, dbl, dbl, _P, _P, _P, _P, i32,
                                  dbl, _P, _P, _P, _P, _P, _P, u32]),
        'acs_sba_ekf_pipeline': (C.c_int, [_P, _P, i64, _P, i64, _P, i32, _P, _P, i32, i32, i32, _P, dbl, dbl, dbl,
                                           _P, _P, _P, C.POINTER(SbaOpts), C.POINTER(EkfInitSpec), i32, dbl, _P, _P,
                                           _P, _P, C.POINTER(Report), u32]),
        'acs_sba_extrinsics': (C.c_int, [_P, _P, i32, _P, _P, _P, i64, _P, i64, C.POINTER(SbaExtOpts), _P, _P,
                                         C.POINTER(SbaExtReport), u32]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def alloc_events():
    """acs_alloc_events: device / pinned-host allocations + frees the library has made in this
    process (no GPU needed)."""
    return int(load_library().acs_alloc_events())


def load_library():
    """Load libacinoset_hip.so (no GPU needed). Raises NativeUnavailable if missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeUnavailable(
                    f'{LIB_PATH} not found: build it with `python -c "import __graft_entry__ as g; g.build()"` '
                    '(hipcc --offload-arch=gfx950). There is no CPU fallback.')
            lib = C.CDLL(LIB_PATH)
            _declare(lib)
            got = lib.acs_abi_version()
            if got != ABI_VERSION:
                raise NativeUnavailable(f'{LIB_PATH} has C ABI version {got}, this package needs {ABI_VERSION} '
                                        '(include/acinoset_hip.h ACS_ABI_VERSION): rebuild the library')
            _lib = lib
    return _lib


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    return C.c_void_p(a.ctypes.data)


def _c64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def pack_cameras(K, D, R, t) -> np.ndarray:
    """(C,3,3),(C,4[,1]),(C,3,3),(C,3[,1]) -> (C, 20) camera records (header: camera block)."""
    K = np.asarray(K, np.float64).reshape(-1, 3, 3)
    n = len(K)
    D = np.asarray(D, np.float64).reshape(n, 4)
    R = np.asarray(R, np.float64).reshape(n, 3, 3)
    t = np.asarray(t, np.float64).reshape(n, 3)
    cams = np.empty((n, ACS_CAM_STRIDE))
    cams[:, 0] = K[:, 0, 0]
    cams[:, 1] = K[:, 1, 1]
    cams[:, 2] = K[:, 0, 2]
    cams[:, 3] = K[:, 1, 2]
    cams[:, 4:8] = D
    cams[:, 8:17] = R.reshape(n, 9)
    cams[:, 17:20] = t
    return cams


class Context:
    """One HIP device + stream (acs_ctx). Methods take numpy arrays (host pointers)
    unless `device_ptrs=True`, in which case they take raw device addresses (ints)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _P()
        rc = self.lib.acs_ctx_create(int(device), C.byref(h))
        if rc != 0:
            n = C.c_int(0)
            self.lib.acs_device_count(C.byref(n))
            raise NativeUnavailable(f'acs_ctx_create(device={device}) failed with {rc}: {n.value} HIP device(s) '
                                    'visible; a gfx950 (MI355X) device is required and there is no CPU fallback.')
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, 'h', None):
            self.lib.acs_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc, what):
        if rc != 0:
            msg = self.lib.acs_last_error(self.h)
            raise RuntimeError(f'{what} failed ({rc}): {msg.decode() if msg else ""}')

    def set_stream(self, stream_handle: int):
        self.check(self.lib.acs_ctx_set_stream(self.h, C.c_void_p(stream_handle or 0)), 'acs_ctx_set_stream')

    def sync(self):
        self.check(self.lib.acs_ctx_sync(self.h), 'acs_ctx_sync')

    # ---- a1 -------------------------------------------------------------------------
    def project(self, cams, pts, cam_idx=None, fte_form=False):
        cams = _c64(cams)
        pts = _c64(pts).reshape(-1, 3)
        n = len(pts)
        ci = None if cam_idx is None else np.ascontiguousarray(np.broadcast_to(cam_idx, (n,)), np.int32)
        out = np.empty((n, 2))
        self.check(self.lib.acs_project_fisheye(self.h, _ptr(cams), len(cams), _ptr(pts), _ptr(ci), n,
                                                int(bool(fte_form)), _ptr(out), 0), 'acs_project_fisheye')
        return out

    # ---- a2 -------------------------------------------------------------------------
    def sba_residuals(self, cams, uv, pt_idx, cam_idx, pts):
        cams = _c64(cams)
        uv = _c64(uv).reshape(-1, 2)
        pi = np.ascontiguousarray(pt_idx, np.int32)
        ci = np.ascontiguousarray(cam_idx, np.int32)
        pts = _c64(pts).reshape(-1, 3)
        out = np.empty(2 * len(uv))
        self.check(self.lib.acs_sba_residuals(self.h, _ptr(cams), len(cams), _ptr(uv), _ptr(pi), _ptr(ci), len(uv),
                                              _ptr(pts), len(pts), _ptr(out), 0), 'acs_sba_residuals')
        return out

    # ---- a4 -------------------------------------------------------------------------
    @staticmethod
    def sba_opts(f_scale=50.0, max_iters=100, ftol=1e-15, xtol=1e-9, gtol=1e-10):
        return SbaOpts(int(max_iters), 0, float(f_scale), float(ftol), float(xtol), float(gtol))

    def sba_points(self, cams, uv, pt_idx, cam_idx, pts0, opts=None, residuals=True):
        cams = _c64(cams)
        uv = _c64(uv).reshape(-1, 2)
        pi = np.ascontiguousarray(pt_idx, np.int32)
        ci = np.ascontiguousarray(cam_idx, np.int32)
        pts = _c64(pts0).reshape(-1, 3).copy()
        rb = np.empty(2 * len(uv)) if residuals else None
        ra = np.empty(2 * len(uv)) if residuals else None
        rep = Report()
        opts = opts or self.sba_opts()
        self.check(self.lib.acs_sba_points(self.h, _ptr(cams), len(cams), _ptr(uv), _ptr(pi), _ptr(ci), len(uv),
                                           _ptr(pts), len(pts), C.byref(opts), _ptr(rb), _ptr(ra), C.byref(rep), 0),
                   'acs_sba_points')
        return pts, rb, ra, rep.as_dict()

    def sba_points_dense(self, cams, uv, mask, pts0, opts=None):
        cams = _c64(cams)
        C_ = len(cams)
        uv = _c64(uv).reshape(-1, C_, 2)
        mask = np.ascontiguousarray(mask, np.uint8).reshape(-1, C_)
        pts = _c64(pts0).reshape(-1, 3).copy()
        rep = Report()
        opts = opts or self.sba_opts()
        self.check(self.lib.acs_sba_points_dense(self.h, _ptr(cams), C_, _ptr(uv), _ptr(mask), len(pts), _ptr(pts),
                                                 C.byref(opts), C.byref(rep), 0), 'acs_sba_points_dense')
        return pts, rep.as_dict()

    def sba_points_dense_dev(self, cams_p, n_cams, uv_p, mask_p, n_pts, pts_p, opts=None, report=False,
                             pts_in_p=None):
        """Device-pointer variant (inputs resident in HBM; asynchronous unless report).
        With `pts_in_p` the initial points are read from there and the solution written
        to `pts_p` (acs_sba_points_dense_io); otherwise `pts_p` is in/out."""
        opts = opts or self.sba_opts()
        rep = Report() if report else None
        rp = C.byref(rep) if rep is not None else None
        if pts_in_p is None:
            rc = self.lib.acs_sba_points_dense(self.h, C.c_void_p(cams_p), n_cams, C.c_void_p(uv_p),
                                               C.c_void_p(mask_p), n_pts, C.c_void_p(pts_p), C.byref(opts), rp,
                                               ACS_DEVICE_PTRS)
        else:
            rc = self.lib.acs_sba_points_dense_io(self.h, C.c_void_p(cams_p), n_cams, C.c_void_p(uv_p),
                                                  C.c_void_p(mask_p), n_pts, C.c_void_p(pts_in_p),
                                                  C.c_void_p(pts_p), C.byref(opts), rp, ACS_DEVICE_PTRS)
        self.check(rc, 'acs_sba_points_dense')
        return rep.as_dict() if rep is not None else None

    # ---- a6 -------------------------------------------------------------------------
    def sba_ext_opts(self, **kw):
        o = SbaExtOpts()
        self.lib.acs_sba_ext_default_opts(C.byref(o))
        for k, v in kw.items():
            setattr(o, k, v)
        return o

    def sba_extrinsics(self, cams, uv, pt_idx, cam_idx, pts0, opts=None, residuals=True):
        """Points + camera extrinsics LM. Returns (cams (C,20), pts (n,3), res_before, res_after, report)."""
        cams = _c64(cams).copy()
        uv = _c64(uv).reshape(-1, 2)
        pi = np.ascontiguousarray(pt_idx, np.int32)
        ci = np.ascontiguousarray(cam_idx, np.int32)
        pts = _c64(pts0).reshape(-1, 3).copy()
        rb = np.empty(2 * len(uv)) if residuals else None
        ra = np.empty(2 * len(uv)) if residuals else None
        rep = SbaExtReport()
        opts = opts or self.sba_ext_opts()
        self.check(self.lib.acs_sba_extrinsics(self.h, _ptr(cams), len(cams), _ptr(uv), _ptr(pi), _ptr(ci), len(uv),
                                               _ptr(pts), len(pts), C.byref(opts), _ptr(rb), _ptr(ra),
                                               C.byref(rep), 0), 'acs_sba_extrinsics')
        return cams, pts, rb, ra, rep.as_dict()

    # ---- f2: EKF + RTS smoother ----------------------------------------------------------
    def ekf_run(self, table, cams, meas, likelihood, fps, thresh, max_pixel_err, r_std_base, Q, P0, s0,
                ref_numerics=True, eps=1e-3, covariances=False, jacobian='fd'):
        """meas (S, N, C, L, 2) or (N, C, L, 2); returns dict of x_pred, x_est, x_smooth
        (S, N, n) [, P_est, P_smooth (S, N, n, n)], outliers (S,)."""
        cams = _c64(cams)
        meas = _c64(meas)
        single = meas.ndim == 4
        if single:
            meas = meas[None]
        S, N, Cn, L, _ = meas.shape
        assert L == table.L and Cn == len(cams), (meas.shape, table.L, len(cams))
        lik = _c64(likelihood).reshape(S, N, Cn, L)
        n = 3 * table.P
        s0 = _c64(s0).reshape(S, n)
        out = {k: np.empty((S, N, n)) for k in ('x_pred', 'x_est', 'x_smooth')}
        if covariances:
            out.update(P_est=np.empty((S, N, n, n)), P_smooth=np.empty((S, N, n, n)))
        outl = np.zeros(S, np.int64)
        ints = np.ascontiguousarray(table.ints, np.int32)
        reals = np.ascontiguousarray(table.reals, np.float64)
        self.check(self.lib.acs_ekf_run(self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(cams), Cn,
                                        _ptr(meas), _ptr(lik), S, N, float(fps), float(thresh), float(max_pixel_err),
                                        _ptr(_c64(r_std_base)), _ptr(_c64(Q)), _ptr(_c64(P0)), _ptr(s0),
                                        ekf_numerics_mode(ref_numerics, jacobian), float(eps), _ptr(out['x_pred']), _ptr(out['x_est']),
                                        _ptr(out['x_smooth']), _ptr(out.get('P_est')), _ptr(out.get('P_smooth')),
                                        _ptr(outl), 0), 'acs_ekf_run')
        out['outliers'] = outl
        if single:
            out = {k: v[0] for k, v in out.items()}
        return out

    def ekf_run_dev(self, ints_p, n_ints, reals_p, n_reals, cams_p, n_cams, meas_p, lik_p, S, N, fps, thresh,
                    max_pixel_err, r_std_p, Q_p, P0_p, s0_p, x_est_p, x_smooth_p, x_pred_p=None, ref_numerics=True,
                    eps=1e-3, jacobian='fd'):
        """acs_ekf_run on device pointers (ACS_DEVICE_PTRS: inputs resident in HBM, outputs
        written there; asynchronous on the context stream, no outliers report): the layouts of
        ekf_run, every pointer an int (torch data_ptr()). Being asynchronous, the call does not
        check for singular solves itself: read them afterwards with ekf_singular_count()."""
        v = lambda p: C.c_void_p(p) if p else None  # noqa: E731
        self.check(self.lib.acs_ekf_run(self.h, v(ints_p), n_ints, v(reals_p), n_reals, v(cams_p), n_cams, v(meas_p),
                                        v(lik_p), S, N, float(fps), float(thresh), float(max_pixel_err), v(r_std_p),
                                        v(Q_p), v(P0_p), v(s0_p), ekf_numerics_mode(ref_numerics, jacobian),
                                        float(eps), v(x_pred_p), v(x_est_p), v(x_smooth_p), None, None, None,
                                        ACS_DEVICE_PTRS), 'acs_ekf_run')

    def ekf_singular_count(self):
        """Singular solves of the last EKF enqueue on this context (waits for its stream)."""
        n = C.c_int32(0)
        self.check(self.lib.acs_ekf_singular_count(self.h, C.byref(n)), 'acs_ekf_singular_count')
        return int(n.value)

    # ---- configs[4]: SBA + EKF fused ------------------------------------------------
    def sba_ekf_pipeline(self, table, cams, meas, likelihood, obs_markers, fps, thresh, max_pixel_err, r_std_base, Q,
                         P0, sba_opts=None, from_sba=False, ref_numerics=True, eps=1e-3, jacobian='fd'):
        """acs_sba_ekf_pipeline on host arrays: meas (S, N, C, Lobs, 2), likelihood (S, N, C,
        Lobs) with markers `obs_markers`; the EKF runs skeleton `table` (its markers a subset of
        obs_markers). Returns dict pts (S, N, Lobs, 3), x_est, x_smooth (S, N, 3P), outliers
        (S,), sba (report dict)."""
        cams = _c64(cams)
        meas = _c64(meas)
        S, N, Cn, Lo, _ = meas.shape
        assert Lo == len(obs_markers) and Cn == len(cams), (meas.shape, len(obs_markers), len(cams))
        lik = _c64(likelihood).reshape(S, N, Cn, Lo)
        obs = list(obs_markers)
        emap = np.array([obs.index(m) for m in table.markers], np.int32)
        n = 3 * table.P
        pts = np.empty((S, N, Lo, 3))
        xe = np.empty((S, N, n))
        xs = np.empty((S, N, n))
        outl = np.zeros(S, np.int64)
        rep = Report()
        opts = sba_opts or self.sba_opts()
        spec = ekf_init_spec(table, obs, from_sba)
        ints = np.ascontiguousarray(table.ints, np.int32)
        reals = np.ascontiguousarray(table.reals, np.float64)
        self.check(self.lib.acs_sba_ekf_pipeline(
            self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(cams), Cn, _ptr(meas), _ptr(lik), S, N, Lo,
            _ptr(emap), float(fps), float(thresh), float(max_pixel_err), _ptr(_c64(r_std_base)), _ptr(_c64(Q)),
            _ptr(_c64(P0)), C.byref(opts), C.byref(spec), ekf_numerics_mode(ref_numerics, jacobian), float(eps), _ptr(pts), _ptr(xe),
            _ptr(xs), _ptr(outl), C.byref(rep), 0), 'acs_sba_ekf_pipeline')
        return dict(pts=pts, x_est=xe, x_smooth=xs, outliers=outl, sba=rep.as_dict())

    def sba_ekf_pipeline_dev(self, table, obs_markers, cams_p, n_cams, meas_p, lik_p, S, N, fps, thresh,
                             max_pixel_err, rstd_p, Q_p, P0_p, pts_p, xe_p, xs_p, sba_opts=None, from_sba=False,
                             ref_numerics=True, eps=1e-3, report=False, jacobian='fd'):
        """acs_sba_ekf_pipeline on HBM-resident arrays (device pointers, asynchronous unless
        `report`: then waits and returns (sba report dict, outliers (S,)))."""
        obs = list(obs_markers)
        emap = np.array([obs.index(m) for m in table.markers], np.int32)
        spec = ekf_init_spec(table, obs, from_sba)
        opts = sba_opts or self.sba_opts()
        ints = np.ascontiguousarray(table.ints, np.int32)
        reals = np.ascontiguousarray(table.reals, np.float64)
        rep = Report() if report else None
        outl = np.zeros(S, np.int64) if report else None
        P_ = C.c_void_p
        self.check(self.lib.acs_sba_ekf_pipeline(
            self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), P_(cams_p), n_cams, P_(meas_p), P_(lik_p), S, N,
            len(obs), _ptr(emap), float(fps), float(thresh), float(max_pixel_err), P_(rstd_p), P_(Q_p), P_(P0_p),
            C.byref(opts), C.byref(spec), ekf_numerics_mode(ref_numerics, jacobian), float(eps), P_(pts_p), P_(xe_p), P_(xs_p),
            _ptr(outl), C.byref(rep) if report else None, ACS_DEVICE_PTRS), 'acs_sba_ekf_pipeline')
        return (rep.as_dict(), outl) if report else None

    # ---- a9 -------------------------------------------------------------------------
    def redescending_loss(self, err, a=3.0, b=10.0, c=20.0, deriv=False):
        e = _c64(err).ravel()
        out = np.empty_like(e)
        d = np.empty_like(e) if deriv else None
        self.check(self.lib.acs_redescending_loss(self.h, _ptr(e), len(e), a, b, c, _ptr(out), _ptr(d), 0),
                   'acs_redescending_loss')
        return (out, d) if deriv else out

    # ---- a7 -------------------------------------------------------------------------
    def fk(self, table, x, dx=None, ddx=None, tau=None, intermode=0, directions=False, jac=False):
        x = _c64(x).reshape(-1, table.P)
        n = len(x)
        dx = None if dx is None else _c64(dx).reshape(n, table.P)
        ddx = None if ddx is None else _c64(ddx).reshape(n, table.P)
        tau = None if tau is None else _c64(np.broadcast_to(tau, (n,)))
        Lo = table.L + (2 if directions else 0)
        out = np.empty((n, Lo, 3))
        J = np.empty((n, table.L, 3, table.P)) if jac else None
        ints = np.ascontiguousarray(table.ints, np.int32)
        reals = np.ascontiguousarray(table.reals, np.float64)
        self.check(self.lib.acs_fk(self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(x), _ptr(dx),
                                   _ptr(ddx), _ptr(tau), n, int(intermode), int(bool(directions)), _ptr(out),
                                   _ptr(J), 0), 'acs_fk')
        return (out, J) if jac else out

    # ---- a10-a13: FTE ------------------------------------------------------------------
    def fte_default_opts(self, **kw):
        o = FteOpts()
        self.lib.acs_fte_default_opts(C.byref(o))
        for k, v in kw.items():
            setattr(o, k, v)
        return o

    def _fte_args(self, table, cams, meas, w, Ts, qinv, shutter_delay, intermode):
        cams = _c64(cams)
        N, Cn, L, _ = np.shape(meas)
        assert L == table.L and Cn == len(cams), (np.shape(meas), table.L, len(cams))
        meas = _c64(np.nan_to_num(meas))
        w = _c64(w).reshape(N, Cn, L)
        qinv = _c64(qinv).reshape(table.P)
        ints = np.ascontiguousarray(table.ints, np.int32)
        reals = np.ascontiguousarray(table.reals, np.float64)
        return ints, reals, cams, meas, w, qinv, N, Cn

    @staticmethod
    def _tau_init(tau, N, Cn, sd_mode):
        """Shutter delays in the layout of sd_mode (0 const: (C,), 1 variable: (N, C)),
        camera 0 pinned at 0 (src/core/fte.py:304-308)."""
        shape = (N, Cn) if sd_mode == 1 else (Cn,)
        t = np.zeros(shape) if tau is None else np.array(np.broadcast_to(_c64(tau), shape), np.float64)
        t[..., 0] = 0.0
        return np.ascontiguousarray(t)

    def fte_solve(self, table, cams, meas, w, Ts, qinv, X0, tau0=None, shutter_delay=True, intermode=1,
                  opts=None, sd_mode=0):
        """sd_mode 0 = 'const' (tau (C,)), 1 = 'variable' (tau (N, C), src/core/fte.py:236-238)."""
        ints, reals, cams, meas, w, qinv, N, Cn = self._fte_args(table, cams, meas, w, Ts, qinv, shutter_delay,
                                                                 intermode)
        sd_mode = SD_MODES.get(sd_mode, sd_mode)
        X = _c64(X0).reshape(N + 2, table.P).copy()
        tau = self._tau_init(tau0, N, Cn, sd_mode)
        rep = FteReport()
        opts = opts or self.fte_default_opts()
        self.check(self.lib.acs_fte_solve(self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(cams), Cn,
                                          _ptr(meas), _ptr(w), N, int(bool(shutter_delay)), float(Ts), _ptr(qinv),
                                          int(sd_mode), int(intermode), _ptr(X), _ptr(tau), C.byref(opts),
                                          C.byref(rep), 0), 'acs_fte_solve')
        return X, tau, rep.as_dict()

    def fte_solve_dev(self, table_ints_p, n_ints, table_reals_p, n_reals, cams_p, n_cams, meas_p, w_p, N,
                      shutter_delay, Ts, qinv_p, intermode, X_p, tau_p, opts=None, sd_mode=0):
        """Device-pointer variant (all arrays resident in HBM); returns the report."""
        sd_mode = SD_MODES.get(sd_mode, sd_mode)
        rep = FteReport()
        opts = opts or self.fte_default_opts()
        self.check(self.lib.acs_fte_solve(self.h, C.c_void_p(table_ints_p), n_ints, C.c_void_p(table_reals_p), n_reals,
                                          C.c_void_p(cams_p), n_cams, C.c_void_p(meas_p), C.c_void_p(w_p), N,
                                          int(bool(shutter_delay)), float(Ts), C.c_void_p(qinv_p), int(sd_mode),
                                          int(intermode),
                                          C.c_void_p(X_p), C.c_void_p(tau_p), C.byref(opts), C.byref(rep),
                                          ACS_DEVICE_PTRS), 'acs_fte_solve')
        return rep.as_dict()

    def fte_eval(self, table, cams, meas, w, Ts, qinv, X, tau=None, shutter_delay=True, intermode=1, hessian=True,
                 sd_mode=0):
        ints, reals, cams, meas, w, qinv, N, Cn = self._fte_args(table, cams, meas, w, Ts, qinv, shutter_delay,
                                                                 intermode)
        sd_mode = SD_MODES.get(sd_mode, sd_mode)
        X = _c64(X).reshape(N + 2, table.P)
        tau = np.zeros((N, Cn) if sd_mode == 1 else Cn) if tau is None else _c64(tau)
        nv = (N + 2) * table.P + ((N * Cn if sd_mode == 1 else Cn) if shutter_delay else 0)
        cost = np.empty(3)
        grad = np.empty(nv)
        H = np.empty((nv, nv)) if hessian else None
        self.check(self.lib.acs_fte_eval(self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(cams), Cn,
                                         _ptr(meas), _ptr(w), N, int(bool(shutter_delay)), float(Ts), _ptr(qinv),
                                         int(sd_mode), int(intermode), _ptr(X), _ptr(tau), _ptr(cost), _ptr(grad),
                                         _ptr(H), 0),
                   'acs_fte_eval')
        return cost, grad, H

    def fte_debug_blocks(self, table, cams, meas, w, Ts, qinv, X, tau=None, lam=0.0, levels=0, shutter_delay=True,
                         intermode=1):
        """acs_fte_debug_blocks (test hook): the damped super-blocks D (n_blk, BP, BP) of the FTE's
        block-tridiagonal system at (X, tau), after `levels` cyclic-reduction levels with the
        pending Schur terms applied (blocks 2^levels m then hold the D the next level factors).
        Returns (D, levels run)."""
        ints, reals, cams, meas, w, qinv, N, Cn = self._fte_args(table, cams, meas, w, Ts, qinv, shutter_delay,
                                                                 intermode)
        X = _c64(X).reshape(N + 2, table.P)
        tau = self._tau_init(tau, N, Cn, 0)
        nblk = (N + 2 + 2) // 3
        BP = ((3 * table.P + 15) // 16) * 16
        D = np.empty((nblk, BP, BP))
        dims = (C.c_int64 * 3)()
        self.check(self.lib.acs_fte_debug_blocks(self.h, _ptr(ints), len(ints), _ptr(reals), len(reals), _ptr(cams), Cn,
                                                 _ptr(meas), _ptr(w), N, int(bool(shutter_delay)), float(Ts),
                                                 _ptr(qinv), 0, int(intermode), _ptr(X), _ptr(tau), float(lam),
                                                 int(levels), _ptr(D), dims, 0), 'acs_fte_debug_blocks')
        assert dims[0] == nblk and dims[1] == BP, (list(dims), nblk, BP)
        return D, int(dims[2])

    # ---- triangulation -------------------------------------------------
    def triangulate_pairs(self, cams, uv_a, uv_b, cam_a, cam_b):
        cams = _c64(cams)
        uv_a = _c64(uv_a).reshape(-1, 2)
        uv_b = _c64(uv_b).reshape(-1, 2)
        n = len(uv_a)
        ca = np.ascontiguousarray(np.broadcast_to(cam_a, (n,)), np.int32)
        cb = np.ascontiguousarray(np.broadcast_to(cam_b, (n,)), np.int32)
        out = np.empty((n, 3))
        self.check(self.lib.acs_triangulate_pairs(self.h, _ptr(cams), len(cams), _ptr(uv_a), _ptr(uv_b), _ptr(ca),
                                                  _ptr(cb), n, _ptr(out), 0), 'acs_triangulate_pairs')
        return out

    def triangulate_dense(self, cams, uv, mask):
        cams = _c64(cams)
        C_ = len(cams)
        uv = _c64(np.nan_to_num(uv)).reshape(-1, C_, 2)
        mask = np.ascontiguousarray(mask, np.uint8).reshape(-1, C_)
        n = len(uv)
        out = np.empty((n, 3))
        cnt = np.empty(n, np.int32)
        self.check(self.lib.acs_triangulate_dense(self.h, _ptr(cams), C_, _ptr(uv), _ptr(mask), n, _ptr(out),
                                                  _ptr(cnt), 0), 'acs_triangulate_dense')
        return out, cnt


_default_ctx = None


def default_context() -> Context:
    """Process-wide context on the device selected by LOCAL_RANK (default 0)."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get('ACINOSET_DEVICE', os.environ.get('LOCAL_RANK', 0))))
    return _default_ctx
