"""Multi-GPU solves of the hot path: frame-window FTE (BASELINE
configs[3]) and points + extrinsics SBA with a reduced-camera-system all-reduce.

Frame-window FTE:

One process per GPU (torchrun); ranks split the trajectory's 3-frame super-blocks into
chains that share their end blocks (include/acinoset_hip.h, acs_fte_dist_*). Every LM
step is ONE all-reduce (sum) of one payload: the chain ends' reduced normal-equation blocks +
tau border (~1 MB at 8 ranks) and the previous step's trial cost and step / state norms (4
doubles), with `torch.distributed.all_reduce` (RCCL over xGMI on the "nccl" backend; gloo in
the CPU tests). A round, on the summed payload: every rank takes the same accept / reject
decision on the pending step, runs the same reduced solve, back-substitutes and steps its
own chain (X lives on the chain only: the terms a rank owns never read other rows), and
packs the new step's cost and the reduced system at its trial state - formed speculatively
with the damping an acceptance gives; a rejected step costs one extra round that re-forms
the reduced system at the unchanged state. Decisions are taken on the device and the host
reads a round's status one round late (`poll`), so the next round and its all-reduce are
queued before the previous one has finished. The solution rows (n_blocks x BP) cross the
ranks once, after the last round.

`lm_loop` is the protocol, independent of the backend: the HIP ranks below, or the numpy
restatement in oracle/fte_dist.py that the CPU tests plug in.

Points + extrinsics SBA (`lm_loop` too): points are split over the ranks, cameras
replicated; per LM step ONE all-reduce of one payload: the reduced camera system
(6C x 6C + vectors, 11 KB at C = 6) formed speculatively at the trial state, and that
trial's cost / step norms (3 doubles), with the same decide / step / re-form round as the
frame-window FTE.
"""
import ctypes as C

import numpy as np

from . import _native


def lm_loop(ranks, allreduce):
    """Drive the distributed LM. `ranks`: the backends living in this process (one per
    process under torch.distributed, several for the single-process emulation);
    `allreduce(list_of_payloads)` sums the i-th payload over all ranks in place.
    One all-reduce per round; round k's status is read after round k + 1 is queued (a
    round after the stop is a no-op on every rank). Returns the final status."""
    P = [r.init() for r in ranks]
    allreduce(P)
    k = 0
    while True:
        P = [r.round(p) for r, p in zip(ranks, P)]
        allreduce(P)
        if k >= 1:
            st = [r.poll(k - 1) for r in ranks]
            assert len(set(st)) == 1, f'ranks diverged: {st}'
            if st[0] != 0:
                break
        k += 1
    if hasattr(ranks[0], 'gather'):
        # frame-window FTE: the solution rows of every chain, once
        p2 = [r.gather() for r in ranks]
        allreduce(p2)
        for r, a in zip(ranks, p2):
            r.scatter(a)
    return st[0]


def _check_dev(torch, dev, device, table, N, Cn, var=False):
    """The HBM-resident inputs of a rank go to the C ABI as raw pointers: check what the
    kernels assume (device, dtype, contiguity, element counts) before handing them over."""
    want = {'ints': (torch.int32, len(table.ints)), 'reals': (torch.float64, len(table.reals)),
            'cams': (torch.float64, Cn * _native.ACS_CAM_STRIDE), 'meas': (torch.float64, N * Cn * table.L * 2),
            'w': (torch.float64, N * Cn * table.L), 'qinv': (torch.float64, table.P),
            'X': (torch.float64, (N + 2) * table.P), 'tau': (torch.float64, N * Cn if var else Cn)}
    for k, (dt, n) in want.items():
        t = dev.get(k)
        if t is None:
            raise ValueError(f'dev[{k!r}] missing')
        if t.device.type != 'cuda' or t.device.index != device:
            raise ValueError(f'dev[{k!r}] is on {t.device}, the context is on cuda:{device}')
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError(f'dev[{k!r}] must be a contiguous {dt} tensor (got {t.dtype}, '
                             f'contiguous={t.is_contiguous()})')
        if t.numel() != n:
            raise ValueError(f'dev[{k!r}] has {t.numel()} elements, expected {n}')


class HipFteRank:
    """One rank of the distributed solve on a HIP context (payloads are torch device
    tensors, so torch.distributed can reduce them in place)."""

    def __init__(self, ctx, table, cams, meas, w, Ts, qinv, X0, tau0=None, shutter_delay=True, intermode=1,
                 opts=None, rank=0, world=1, dev=None, sd_mode=0):
        """`dev`: the inputs already resident in HBM, as torch device tensors
        {'ints', 'reals', 'cams', 'meas', 'w', 'qinv', 'X', 'tau'} (copied device to device
        into the handle; the host arrays are then only used for the shapes). sd_mode 0 =
        'const' (tau (C,)), 1 = 'variable' (tau (N, C): each frame's delays eliminated and
        stepped by the rank owning the frame, gathered with the solution rows)."""
        import torch
        self.ctx = ctx
        self.torch = torch
        opts = opts or ctx.fte_default_opts()
        sd_mode = _native.SD_MODES.get(sd_mode, sd_mode)
        h = C.c_void_p()
        sizes = (C.c_int64 * 3)()
        if dev is None:
            ints, reals, cams, meas, w, qinv, N, Cn = ctx._fte_args(table, cams, meas, w, Ts, qinv, shutter_delay,
                                                                    intermode)
            X = _native._c64(X0).reshape(N + 2, table.P)
            tau = ctx._tau_init(tau0, N, Cn, sd_mode if shutter_delay else 0)
            P_ = _native._ptr
            ptrs = [P_(a) for a in (ints, reals, cams, meas, w, qinv, X, tau)]
            n_ints, n_reals, flags = len(ints), len(reals), 0
        else:
            N, Cn = int(np.shape(meas)[0]), int(np.shape(meas)[1])
            _check_dev(torch, dev, ctx.device, table, N, Cn, sd_mode == 1 and shutter_delay)
            ptrs = [C.c_void_p(dev[k].data_ptr()) for k in ('ints', 'reals', 'cams', 'meas', 'w', 'qinv', 'X', 'tau')]
            n_ints, n_reals, flags = dev['ints'].numel(), dev['reals'].numel(), _native.ACS_DEVICE_PTRS
        self.N, self.P, self.C = N, table.P, Cn
        self.tau_shape = (N, Cn) if (sd_mode == 1 and shutter_delay) else (Cn,)
        ctx.check(ctx.lib.acs_fte_dist_create(ctx.h, ptrs[0], n_ints, ptrs[1], n_reals, ptrs[2], Cn, ptrs[3], ptrs[4], N,
                                              int(bool(shutter_delay)), float(Ts), ptrs[5], int(sd_mode),
                                              int(intermode), ptrs[6], ptrs[7], C.byref(opts), int(rank), int(world),
                                              C.byref(h), sizes, flags),
                  'acs_fte_dist_create')
        self.h = h
        dev = torch.device('cuda', ctx.device)
        # two round payloads (a round reads one and writes the other) and the solution rows
        self.bufs = [torch.zeros(int(sizes[0]), dtype=torch.float64, device=dev) for _ in range(2)]
        self.p2 = torch.zeros(int(sizes[1]), dtype=torch.float64, device=dev)
        self.which = 0

    def _ptr(self, t):
        return C.c_void_p(t.data_ptr())

    def reset(self, X0, tau0=None):
        """Restart the solve on this handle from X0 ((N + 2, P)) and tau0 (None = zeros): host
        arrays, or torch device tensors on the context's device (ACS_DEVICE_PTRS). No
        allocation: the arena, payloads and captured round graphs are reused
        (acs_fte_dist_reset), so a timed multi-GPU solve creates its ranks once."""
        torch = self.torch
        if isinstance(X0, torch.Tensor):
            for t, n in ((X0, (self.N + 2) * self.P), (tau0, int(np.prod(self.tau_shape)))):
                if t is None:
                    continue
                if (t.device.type != 'cuda' or t.device.index != self.ctx.device or t.dtype != torch.float64
                        or not t.is_contiguous() or t.numel() != n):
                    raise ValueError(f'reset: a contiguous float64 cuda:{self.ctx.device} tensor of {n} elements '
                                     f'expected, got {t.dtype} {tuple(t.shape)} on {t.device}')
            tp = self._ptr(tau0) if tau0 is not None else None
            self.ctx.check(self.ctx.lib.acs_fte_dist_reset(self.h, self._ptr(X0), tp, _native.ACS_DEVICE_PTRS),
                           'acs_fte_dist_reset')
        else:
            X = _native._c64(X0).reshape(self.N + 2, self.P)
            tau = None if tau0 is None else _native._c64(tau0).reshape(self.tau_shape)
            self.ctx.check(self.ctx.lib.acs_fte_dist_reset(self.h, _native._ptr(X),
                                                           _native._ptr(tau) if tau is not None else None, 0),
                           'acs_fte_dist_reset')
        self.which = 0

    def init(self):
        self.which = 0
        self.ctx.check(self.ctx.lib.acs_fte_dist_init(self.h, self._ptr(self.bufs[0])), 'acs_fte_dist_init')
        return self.bufs[0]

    def round(self, pin):
        out = self.bufs[self.which ^ 1]
        self.ctx.check(self.ctx.lib.acs_fte_dist_round(self.h, self._ptr(pin), self._ptr(out)), 'acs_fte_dist_round')
        self.which ^= 1
        return out

    def poll(self, k):
        st = C.c_int32(0)
        self.ctx.check(self.ctx.lib.acs_fte_dist_poll(self.h, int(k), C.byref(st)), 'acs_fte_dist_poll')
        return st.value

    def gather(self):
        self.ctx.check(self.ctx.lib.acs_fte_dist_gather(self.h, self._ptr(self.p2)), 'acs_fte_dist_gather')
        return self.p2

    def scatter(self, p2):
        self.ctx.check(self.ctx.lib.acs_fte_dist_scatter(self.h, self._ptr(p2)), 'acs_fte_dist_scatter')

    def result(self, X_out=None, tau_out=None):
        """(X, tau, report). With torch device tensors X_out / tau_out the solution is copied
        into them on the device (ACS_DEVICE_PTRS) and they are returned instead of host arrays."""
        rep = _native.FteReport()
        if X_out is not None:
            self.ctx.check(self.ctx.lib.acs_fte_dist_result(self.h, self._ptr(X_out),
                                                            self._ptr(tau_out) if tau_out is not None else None,
                                                            C.byref(rep), _native.ACS_DEVICE_PTRS),
                           'acs_fte_dist_result')
            return X_out, tau_out, rep.as_dict()
        X = np.empty((self.N + 2, self.P))
        tau = np.empty(self.tau_shape)
        self.ctx.check(self.ctx.lib.acs_fte_dist_result(self.h, _native._ptr(X), _native._ptr(tau), C.byref(rep), 0),
                       'acs_fte_dist_result')
        return X, tau, rep.as_dict()

    def close(self):
        if getattr(self, 'h', None):
            self.ctx.lib.acs_fte_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def torch_allreduce(group=None):
    """All-reduce (sum) of this process's single payload over the process group."""
    import torch.distributed as dist

    def f(payloads):
        assert len(payloads) == 1
        dist.all_reduce(payloads[0], op=dist.ReduceOp.SUM, group=group)
    return f


def local_allreduce(payloads):
    """Single-process emulation: sum in rank order, every rank receives the total (numpy
    arrays or torch tensors)."""
    tot = payloads[0] * 1
    for p in payloads[1:]:
        tot = tot + p
    for p in payloads:
        p[...] = tot


class _on_torch_stream:
    """Run the context's kernels and torch's collectives on one explicit stream."""

    def __init__(self, ctx):
        import torch
        self.ctx, self.torch = ctx, torch
        self.stream = torch.cuda.Stream(device=torch.device('cuda', ctx.device))

    def __enter__(self):
        self.cm = self.torch.cuda.stream(self.stream)
        self.cm.__enter__()
        self.ctx.set_stream(self.stream.cuda_stream)
        return self

    def __exit__(self, *exc):
        self.stream.synchronize()
        self.ctx.set_stream(0)
        return self.cm.__exit__(*exc)


def fte_solve_dist(ctx, table, cams, meas, w, Ts, qinv, X0, tau0=None, shutter_delay=True, intermode=1, opts=None,
                   group=None, sd_mode=0):
    """Drop-in for Context.fte_solve under torch.distributed (one rank per GPU): returns
    (X, tau, report), identical on every rank."""
    import torch.distributed as tdist
    rank, world = tdist.get_rank(group), tdist.get_world_size(group)
    with _on_torch_stream(ctx):
        r = HipFteRank(ctx, table, cams, meas, w, Ts, qinv, X0, tau0, shutter_delay, intermode, opts, rank, world,
                       sd_mode=sd_mode)
        try:
            lm_loop([r], torch_allreduce(group))
            return r.result()
        finally:
            r.close()


def fte_solve_virtual(ctx, table, cams, meas, w, Ts, qinv, X0, tau0=None, shutter_delay=True, intermode=1,
                      opts=None, world=2, sd_mode=0):
    """The distributed algorithm with `world` ranks emulated in one process on one device
    (parity tests of the decomposition without a multi-GPU node)."""
    with _on_torch_stream(ctx):
        ranks = [HipFteRank(ctx, table, cams, meas, w, Ts, qinv, X0, tau0, shutter_delay, intermode, opts, r, world,
                            sd_mode=sd_mode) for r in range(world)]
        try:
            lm_loop(ranks, local_allreduce)
            outs = [r.result() for r in ranks]
            for X, tau, _ in outs[1:]:
                assert np.array_equal(X, outs[0][0]) and np.array_equal(tau, outs[0][1])
            return outs[0]
        finally:
            for r in ranks:
                r.close()


class HipSbaExtRank:
    """One rank of the points + extrinsics SBA: its own points (local indices) and their
    observations; cameras (C, 20) replicated."""

    def __init__(self, ctx, cams, uv, pt_idx, cam_idx, pts, opts=None, rank=0, world=1):
        import torch
        self.ctx = ctx
        cams = _native._c64(cams)
        uv = _native._c64(uv).reshape(-1, 2)
        pi = np.ascontiguousarray(pt_idx, np.int32)
        ci = np.ascontiguousarray(cam_idx, np.int32)
        pts = _native._c64(pts).reshape(-1, 3)
        self.n_cams, self.n_pts = len(cams), len(pts)
        opts = opts or ctx.sba_ext_opts()
        h = C.c_void_p()
        sizes = (C.c_int64 * 2)()
        P_ = _native._ptr
        ctx.check(ctx.lib.acs_sba_ext_dist_create(ctx.h, P_(cams), len(cams), P_(uv), P_(pi), P_(ci), len(uv), P_(pts),
                                                  len(pts), C.byref(opts), int(rank), int(world), C.byref(h), sizes,
                                                  0), 'acs_sba_ext_dist_create')
        self.h = h
        dev = torch.device('cuda', ctx.device)
        # two round payloads [p1 | p3]: a round reads one and writes the other
        self.bufs = [torch.zeros(int(sizes[0]), dtype=torch.float64, device=dev) for _ in range(2)]
        self.k = 0

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr())

    def init(self):
        self.ctx.check(self.ctx.lib.acs_sba_ext_dist_init(self.h, self._ptr(self.bufs[0])), 'acs_sba_ext_dist_init')
        self.k = 0
        return self.bufs[0]

    def round(self, payload):
        out = self.bufs[1] if payload.data_ptr() == self.bufs[0].data_ptr() else self.bufs[0]
        self.ctx.check(self.ctx.lib.acs_sba_ext_dist_round(self.h, self._ptr(payload), self._ptr(out)),
                       'acs_sba_ext_dist_round')
        self.k += 1
        return out

    def poll(self, k):
        st = C.c_int32(0)
        self.ctx.check(self.ctx.lib.acs_sba_ext_dist_poll(self.h, int(k), C.byref(st)), 'acs_sba_ext_dist_poll')
        return st.value

    def result(self):
        cams = np.empty((self.n_cams, _native.ACS_CAM_STRIDE))
        pts = np.empty((self.n_pts, 3))
        rep = _native.SbaExtReport()
        self.ctx.check(self.ctx.lib.acs_sba_ext_dist_result(self.h, _native._ptr(cams), _native._ptr(pts),
                                                            C.byref(rep), 0), 'acs_sba_ext_dist_result')
        return cams, pts, rep.as_dict()

    def close(self):
        if getattr(self, 'h', None):
            self.ctx.lib.acs_sba_ext_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def split_points(pt_idx, n_pts, world):
    """Contiguous point shards: (per-rank point ranges, per-rank observation ids, local ids).
    Every rank computes every shard, so a shard the rank solve cannot take (no point, or no
    observation: acs_sba_ext_dist_create needs both) raises the same ValueError on every rank
    before any collective, instead of one rank failing while the others wait in the
    all-reduce."""
    pt_idx = np.asarray(pt_idx)
    if world < 1 or n_pts < world:
        raise ValueError(f'split_points: {n_pts} points over {world} ranks (each rank needs at least one)')
    bounds = [(n_pts * r) // world for r in range(world + 1)]
    shards = []
    for r in range(world):
        lo, hi = bounds[r], bounds[r + 1]
        obs = np.nonzero((pt_idx >= lo) & (pt_idx < hi))[0]
        if len(obs) == 0:
            raise ValueError(f'split_points: rank {r} of {world} (points {lo}..{hi - 1}) has no observation')
        shards.append((lo, hi, obs, pt_idx[obs] - lo))
    return shards


def sba_extrinsics_dist(ctx, cams, uv, pt_idx, cam_idx, pts, opts=None, group=None):
    """Points + extrinsics SBA under torch.distributed: every rank passes the full problem
    and solves its contiguous point shard. Returns (cams, all points, report) on every
    rank (the points are all-gathered once at the end)."""
    import torch
    import torch.distributed as tdist
    rank, world = tdist.get_rank(group), tdist.get_world_size(group)
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    lo, hi, obs, loc = split_points(pt_idx, len(pts), world)[rank]
    with _on_torch_stream(ctx):
        r = HipSbaExtRank(ctx, cams, np.asarray(uv).reshape(-1, 2)[obs], loc, np.asarray(cam_idx)[obs], pts[lo:hi],
                          opts, rank, world)
        try:
            lm_loop([r], torch_allreduce(group))
            c, p, rep = r.result()
        finally:
            r.close()
        full = torch.zeros((len(pts), 3), dtype=torch.float64, device=torch.device('cuda', ctx.device))
        full[lo:hi] = torch.from_numpy(p).to(full.device)
        tdist.all_reduce(full, group=group)
        return c, full.cpu().numpy(), rep


def sba_extrinsics_virtual(ctx, cams, uv, pt_idx, cam_idx, pts, opts=None, world=2):
    """The distributed points + extrinsics SBA with `world` ranks emulated in one process."""
    pts = np.asarray(pts, np.float64).reshape(-1, 3)
    with _on_torch_stream(ctx):
        shards = split_points(pt_idx, len(pts), world)
        ranks = [HipSbaExtRank(ctx, cams, np.asarray(uv).reshape(-1, 2)[obs], loc, np.asarray(cam_idx)[obs],
                               pts[lo:hi], opts, r, world) for r, (lo, hi, obs, loc) in enumerate(shards)]
        try:
            lm_loop(ranks, local_allreduce)
            outs = [r.result() for r in ranks]
        finally:
            for r in ranks:
                r.close()
    for c, _, _ in outs[1:]:
        assert np.array_equal(c, outs[0][0])
    return outs[0][0], np.concatenate([o[1] for o in outs]), outs[0][2]
