"""Slab-decomposed RMT step over G GPUs.

The reference runs one NumPy/Numba process (benchmarks/soft_disc_in_lid_driven.py:206-235);
this module splits the same loop body into 1D row slabs, one per GPU, with librmt's slab
phases (include/rmt.h, rmt_slab_*) doing all arithmetic and the collectives between them
done here:

* ``TorchComm`` -- one slab per process over ``torch.distributed``: RCCL (backend "nccl")
  moves device tensors directly over xGMI; "gloo" stages through host memory (CPU tests,
  and two processes sharing one GPU).
* ``LocalComm`` -- G virtual slabs in one process on one GPU, exchanges are device copies.
  Same phases, same data movement pattern: the bit-exactness tests of the decomposition
  run on a single GPU with it.

Per step: one halo exchange of (u, v, p, X1, X2) (RMT_SLAB_HALO rows; the stencils of the
SL backtrace and the 4 RK4 stages are recomputed on the overlap instead of exchanged per
stage), an allgather of the known bit rows and of the narrow band's rim (index, X1, X2)
for the exact raster-order extrapolation replicated on every slab, two all-to-all
transposes around the fused column DCT -> / eig -> inverse DCT, a 2-row halo of p_c, and
small allgathers of row-tree roots and per-slab scalars (the means and diagnostics).
"""
import ctypes
import math
import os

import numpy as np

from . import _lib as L
from . import functions as F
from .simulation import _wrap_device

HALO = 12           # RMT_SLAB_HALO
SC_N = 16           # scalar block: [0] max|u|^2, [1..10] diag partials, [11] flags,
SC_M2, SC_DIAG, SC_FLAGS, SC_COUNT, SC_ROOT, SC_FIT = 0, 1, 11, 12, 13, 14
BUF = {"u": 0, "v": 1, "p": 2, "X1": 3, "X2": 4, "phi": 5, "J": 6, "pc": 7, "bits": 8,
       "bits_next": 13,
       "rim": 9, "A": 10, "B": 11, "scal": 12}


def even_splits(n, G, minsz=2):
    """Split range(n) into G contiguous parts with even boundaries (row / column pairs of
    the DCT stay together) as balanced as possible."""
    if G < 1 or n < G * minsz:
        raise ValueError(f"cannot split {n} into {G} parts of >= {minsz}")
    s = [0]
    for k in range(1, G):
        b = int(round(k * n / G))
        b -= b & 1
        s.append(b)
    s.append(n)
    for k in range(G):
        if s[k + 1] - s[k] < minsz:
            raise ValueError(f"split {s} has a part smaller than {minsz}")
    return s


# ------------------------------------------------------------------ communicators --
class LocalComm:
    """G virtual ranks in this process (one GPU): every collective is device copies over
    the list of local slabs, in rank order."""

    def __init__(self, G):
        self.G = G
        self.ranks = list(range(G))

    def halo(self, slabs, planes, nrows):
        import torch
        with torch.no_grad():
            for k, s in enumerate(slabs):
                for name in planes:
                    dst, e = s.view(name), s.top_extra(name)
                    if k > 0:                      # rows [r0 - n, r0) from slab k - 1
                        o = slabs[k - 1]
                        a = max(s.r0 - nrows, s.lo)
                        dst[a - s.lo:s.r0 - s.lo].copy_(o.view(name)[a - o.lo:s.r0 - o.lo])
                    if k + 1 < len(slabs):         # rows [r1 + e, r1 + e + n) from slab k + 1
                        o = slabs[k + 1]
                        t = s.r1 + e
                        b = min(t + nrows, s.hi + e)
                        dst[t - s.lo:b - s.lo].copy_(o.view(name)[t - o.lo:b - o.lo])

    def halo_start(self, slabs, planes, nrows):
        self.halo(slabs, planes, nrows)

    def halo_finish(self, handle):
        pass

    def allgather_rows(self, slabs, name):
        for s in slabs:
            dst = s.view(name)
            for o in slabs:
                if o is not s:
                    dst[o.r0:o.r1].copy_(o.view(name)[o.r0:o.r1])

    def allgather(self, tensors):
        import torch
        g = torch.stack([t.reshape(-1) for t in tensors])
        return [g] * len(tensors)

    def allgather_padded(self, tensors, counts, width):
        """tensors[k][:counts[k] * width] of every rank -> (G, cap * width) on every rank."""
        import torch
        cap = max(counts) if counts else 0
        g = torch.zeros((self.G, max(cap, 1) * width), dtype=tensors[0].dtype,
                        device=tensors[0].device)
        for k, t in enumerate(tensors):
            g[k, :counts[k] * width].copy_(t.reshape(-1)[:counts[k] * width])
        return [g] * len(tensors), cap

    def all_to_all(self, sends, recvs, send_splits, recv_splits):
        for m, r in enumerate(recvs):
            ro = 0
            for k, s in enumerate(sends):
                so = sum(send_splits[k][:m])
                n = send_splits[k][m]
                assert n == recv_splits[m][k]
                r.reshape(-1)[ro:ro + n].copy_(s.reshape(-1)[so:so + n])
                ro += n


class TorchComm:
    """One slab per process over torch.distributed (RANK / WORLD_SIZE from the process
    group).  Backend "nccl" is RCCL on ROCm and moves device tensors directly; "gloo"
    stages every exchange through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.G = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ranks = [self.rank]
        self.staged = dist.get_backend(group) != "nccl"

    def _host(self, t):
        return t.cpu() if self.staged else t

    def _back(self, dst, src):
        if src is not dst:
            dst.copy_(src)

    def halo(self, slabs, planes, nrows):
        self.halo_finish(self.halo_start(slabs, planes, nrows))

    def halo_start(self, slabs, planes, nrows):
        """Post the halo sends / receives; the interior work runs before halo_finish.  With
        RCCL the receives land on RCCL's stream and halo_finish only orders the compute
        stream after them (no host wait)."""
        (s,) = slabs
        dist, k = self.dist, self.rank
        ops, post = [], []
        for name in planes:
            v, e = s.view(name), s.top_extra(name)
            # a plane with e extra top rows (the MAC v faces: rows lo .. hi) owns rows
            # [r0, r1 + e); the neighbours' counts match because every slab holds more than
            # `nrows` rows
            if k > 0:
                a = max(s.r0 - nrows, s.lo)
                o = s.r0 + e - s.lo
                snd = self._host(v[o:o + (s.r0 - a)].contiguous())
                rcv = v[a - s.lo:s.r0 - s.lo]
                rb = rcv.cpu() if self.staged else rcv
                ops += [(dist.isend, snd, k - 1), (dist.irecv, rb, k - 1)]
                post.append((rcv, rb))
            if k + 1 < self.G:
                t = s.r1 + e
                b = min(t + nrows, s.hi + e)
                snd = self._host(v[s.r1 - s.lo - (b - t):s.r1 - s.lo].contiguous())
                rcv = v[t - s.lo:b - s.lo]
                rb = rcv.cpu() if self.staged else rcv
                ops += [(dist.isend, snd, k + 1), (dist.irecv, rb, k + 1)]
                post.append((rcv, rb))
        if not ops:
            return None
        if self.staged:
            reqs = [f(t, peer, group=self.group) for f, t, peer in ops]
        else:
            p2p = [dist.P2POp(f, t, peer, group=self.group) for f, t, peer in ops]
            reqs = dist.batch_isend_irecv(p2p)
        return reqs, post

    def halo_finish(self, handle):
        if handle is None:
            return
        reqs, post = handle
        for r in reqs:
            r.wait()
        for rcv, rb in post:
            self._back(rcv, rb)

    def allgather_rows(self, slabs, name):
        import torch
        (s,) = slabs
        v = s.view(name)
        sizes = [s.splits[k + 1] - s.splits[k] for k in range(self.G)]
        mx = max(sizes)
        mine = torch.zeros((mx,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        mine[:s.r1 - s.r0].copy_(v[s.r0:s.r1])
        mine = self._host(mine)
        out = torch.empty(self.G * mine.numel(), dtype=v.dtype, device=mine.device)
        self.dist.all_gather_into_tensor(out, mine.reshape(-1), group=self.group)
        out = out.view((self.G,) + tuple(mine.shape))
        for k in range(self.G):
            if k != self.rank:
                v[s.splits[k]:s.splits[k + 1]].copy_(out[k, :sizes[k]])

    def allgather(self, tensors):
        import torch
        (t,) = tensors
        src = self._host(t.reshape(-1).contiguous())
        out = torch.empty(self.G * src.numel(), dtype=src.dtype, device=src.device)
        self.dist.all_gather_into_tensor(out, src, group=self.group)
        out = out.view(self.G, src.numel())
        return [out.to(t.device) if self.staged else out]

    def allgather_padded(self, tensors, counts, width):
        import torch
        (t,) = tensors
        cap = max(counts) if counts else 0
        mine = torch.zeros(max(cap, 1) * width, dtype=t.dtype, device=t.device)
        n = counts[self.rank] * width
        mine[:n].copy_(t.reshape(-1)[:n])
        mine = self._host(mine)
        out = torch.empty(self.G * mine.numel(), dtype=t.dtype, device=mine.device)
        self.dist.all_gather_into_tensor(out, mine, group=self.group)
        out = out.view(self.G, mine.numel())
        return [out.to(t.device) if self.staged else out], cap

    def all_to_all(self, sends, recvs, send_splits, recv_splits):
        (snd,), (rcv,) = sends, recvs
        src = self._host(snd.reshape(-1)[:sum(send_splits[0])])
        dst = rcv.reshape(-1)[:sum(recv_splits[0])]
        db = dst.cpu() if self.staged else dst
        self.dist.all_to_all_single(db, src, output_split_sizes=list(recv_splits[0]),
                                    input_split_sizes=list(send_splits[0]), group=self.group)
        self._back(dst, db)


# ---------------------------------------------------------------------- one slab --
class Slab:
    """One rmt_slab: rows [r0, r1) resident as [lo, hi); zero-copy torch views of its
    buffers (device memory owned by librmt)."""

    def __init__(self, ctx, params, G, rank, rsplits, csplits):
        self.lib = L.lib()
        rs = (ctypes.c_int * (G + 1))(*rsplits)
        cs = (ctypes.c_int * (G + 1))(*csplits)
        h = ctypes.c_void_p()
        L.check(self.lib.rmt_slab_create(ctx.bind(), ctypes.byref(params), G, rank, rs, cs,
                                         ctypes.byref(h)), "rmt_slab_create")
        self.h = h
        info = (ctypes.c_int * 8)()
        dtc = ctypes.c_double()
        L.check(self.lib.rmt_slab_info(h, info, ctypes.byref(dtc)))
        self.r0, self.r1, self.lo, self.hi, self.c0, self.c1, self.W, _ = list(info)
        self.dt_const = dtc.value
        self.G, self.rank, self.splits, self.csplits = G, rank, list(rsplits), list(csplits)
        self.NY, self.NX = params.ny, params.nx
        self._views = {}

    def __del__(self):
        try:
            self.lib.rmt_slab_destroy(self.h)
        except Exception:
            pass

    def _ptr(self, bid):
        p = ctypes.c_void_p()
        L.check(self.lib.rmt_slab_buffer(self.h, bid, ctypes.byref(p)))
        return p.value

    def view(self, name):
        if name not in self._views:
            torch = F._torch()
            nl, no = self.hi - self.lo, self.r1 - self.r0
            nc = self.c1 - self.c0
            shape = {"bits": (self.NY, self.W), "bits_next": (self.NY, self.W),
                     "rim": (no * self.NX, 3), "A": (no * self.NX,),
                     "B": (self.NY * nc,), "scal": (SC_N,)}.get(name, (nl, self.NX))
            t = _wrap_device(torch, self._ptr(BUF[name]), shape)
            if name in ("bits", "bits_next"):
                t = t.view(torch.int64)
            self._views[name] = t
        return self._views[name]

    def top_extra(self, name):
        return 0

    def a2a_splits(self):
        """element counts: forward send (to m: rows_me x nc_m), forward recv (from k:
        rows_k x nc_me); the backward transpose swaps them"""
        rows = self.r1 - self.r0
        nc = self.c1 - self.c0
        snd = [rows * (self.csplits[m + 1] - self.csplits[m]) for m in range(self.G)]
        rcv = [(self.splits[k + 1] - self.splits[k]) * nc for k in range(self.G)]
        return snd, rcv


# ------------------------------------------------------------------ the whole step --
class DistributedSim:
    """The fused RMT step of rmt_sim (sim.hip), decomposed into G row slabs.

    ``comm`` is a LocalComm (G slabs here) or a TorchComm (this process's slab).  The
    physics parameters are those of ``simulation.Simulation`` (semi-Lagrangian, one disc).
    """

    def __init__(self, N, comm, *, bc_kind, lid, disc, mu_s, kappa, rho_s, eta_s, mu_f,
                 rho_f, w_t, layers, cfl, dt_cap, stress_band=False, detg_clamp=3.0,
                 options=None):
        torch = F._torch()
        self.torch, self.comm, self.N, self.G = torch, comm, N, comm.G
        self.X, self.Y, self.dx, self.dy = F.create_grid(N, N, 1.0, 1.0)
        self.xs = np.ascontiguousarray(self.X[0, :])
        self.ys = np.ascontiguousarray(self.Y[:, 0])
        P = L.rmt_sim_params()
        P.ny = P.nx = N; P.dx = self.dx; P.dy = self.dy
        P.xs = self.xs.ctypes.data; P.ys = self.ys.ctypes.data
        P.scheme = 0; P.bc_kind = bc_kind; P.lid = lid; P.shape = 1
        P.x0, P.y0, P.R = disc
        P.mu_s, P.kappa, P.rho_s, P.eta_s, P.mu_f, P.rho_f = mu_s, kappa, rho_s, eta_s, mu_f, rho_f
        P.w_t = w_t; P.layers = layers; P.cfl = cfl; P.dt_cap = dt_cap
        P.stress_band = int(bool(stress_band)); P.detg_clamp = detg_clamp; P.energies = 0
        self.params, self.cfl = P, cfl
        self.rsplits = even_splits(N, self.G, HALO)
        self.csplits = even_splits(N, self.G, 2)
        if options:
            self.ctx = F._Ctx(N, N, torch.cuda.current_device())
            for k, v in options.items():
                self.ctx.set_option(k, v)
        else:
            self.ctx = F.ctx_for(N, N)
        self.slabs = [Slab(self.ctx, P, self.G, r, self.rsplits, self.csplits)
                      for r in comm.ranks]
        self.dt_const = self.slabs[0].dt_const
        self.t = 0.0
        self.m2 = None
        self.records = []
        self._counts = (ctypes.c_longlong * self.G)()
        # the asynchronous step (no host round trip inside a step): device dt, a fixed rim
        # capacity per slab, the per-step scalars into a device ring read every sync_every
        self.sync_every = 32
        self._dev_dt = False          # the slabs' device dt holds this step's dt
        self._rim_cap = None          # rim entries moved per slab (set from the first count)
        self._min_owned = min(self.rsplits[k + 1] - self.rsplits[k] for k in range(self.G)) * N
        # the next step's extrapolation geometry beside the projection (layers 1 .. 12: the
        # slabs have their second stream)
        self._early_geo = (1 <= layers <= 12 and
                           int(os.environ.get("RMT_SLAB_EARLY_GEO", "1")) != 0)

    # -------------------------------------------------------------- state in / out --
    def set_state(self, **fields):
        """Full (N, N) host arrays -> every slab's resident rows."""
        torch = self.torch
        for name, arr in fields.items():
            a = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float64))
            for s in self.slabs:
                s.view(name).copy_(a[s.lo:s.hi].to(s.view(name).device))
        self.m2 = None

    def gather(self, name):
        """The owned rows of every slab assembled into a full (N, N) host array."""
        torch = self.torch
        torch.cuda.synchronize()
        views = [s.view(name)[s.r0 - s.lo:s.r1 - s.lo].contiguous() for s in self.slabs]
        if isinstance(self.comm, LocalComm):
            return torch.cat(views).cpu().numpy()
        mx = max(self.rsplits[k + 1] - self.rsplits[k] for k in range(self.G))
        pad = torch.zeros((mx, self.N), dtype=torch.float64, device=views[0].device)
        pad[:views[0].shape[0]].copy_(views[0])
        (g,) = self.comm.allgather([pad])
        g = g.reshape(self.G, mx, self.N).cpu().numpy()
        return np.concatenate([g[k, :self.rsplits[k + 1] - self.rsplits[k]]
                               for k in range(self.G)])

    def _call(self, fn, *args):
        for s in self.slabs:
            L.check(getattr(s.lib, fn)(s.h, *args), fn)

    def _scalars(self):
        """(G, SC_N) host array of every slab's scalar block (one host sync)."""
        g = self.comm.allgather([s.view("scal") for s in self.slabs])[0]
        return g.cpu().numpy().reshape(self.G, SC_N)

    # ----------------------------------------------------------------------- step --
    PHASES = ("halo", "advect", "extrapolate", "momentum", "projection", "finish",
              "rk4_stage_kernels", "extrap_chain_kernel")

    def set_profiling(self, on=True):
        """HIP events (torch.cuda.Event on the stream librmt uses) around each phase, and
        librmt's own kernel timers; read with phase_times()."""
        L.check(L.lib().rmt_ctx_set_profiling(self.ctx.h, int(bool(on))))
        self._prof = bool(on)
        self._ms = {k: 0.0 for k in self.PHASES}
        self._nprof = 0

    def phase_times(self):
        return {k: (v, self._nprof) for k, v in self._ms.items()}

    def _mark(self, ev):
        if getattr(self, "_prof", False):
            e = self.torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)

    def step(self, nsteps=1, t_end=math.inf):
        """nsteps steps (stopping at t_end).  With no t_end and no profiling the steps run
        asynchronously (_step_async: bit-identical, no host round trip inside a step);
        RMT_SLAB_SYNC=1 forces the synchronous path."""
        self.ctx.bind()
        comm, S = self.comm, self.slabs
        if self.m2 is None:
            self._call("rmt_slab_begin")
            self.m2 = float(self._scalars()[:, SC_M2].max())
            self._dev_dt = False
        if (math.isinf(t_end) and t_end > 0 and not getattr(self, "_prof", False)
                and not int(os.environ.get("RMT_SLAB_SYNC", "0"))):
            return self._step_async(nsteps)
        self._step_sync(nsteps, t_end)

    def _step_sync(self, nsteps, t_end):
        """The synchronous path: dt on the host, the rim allgathered at its exact counts."""
        comm, S = self.comm, self.slabs
        self._set_dev_dt(False)
        geo = False
        for k in range(nsteps):
            if not (self.t < t_end):
                break
            ev = []
            self._mark(ev)
            m2 = self.m2
            dt = min(self.dt_const, self.cfl * self.dx / (math.sqrt(m2) + 1e-6))
            if self.t + dt > t_end:
                dt = t_end - self.t
            # halo in flight while the rows that need none are advected
            h = comm.halo_start(S, ("u", "v", "p", "X1", "X2"), HALO)
            self._call("rmt_slab_advect_interior", dt)
            comm.halo_finish(h)
            self._mark(ev)
            # advection + exact extrapolation (band replicated on every slab)
            self._call("rmt_slab_advect", dt)
            self._mark(ev)
            if not geo:   # else the plane was gathered with the early geometry
                comm.allgather_rows(S, "bits")
            geo = False
            self._call("rmt_slab_rim_pack")
            counts = [int(c) for c in self._scalars()[:, SC_COUNT]]
            gathered, cap = comm.allgather_padded([s.view("rim") for s in S], counts, 3)
            for k, c in enumerate(counts):
                self._counts[k] = c
            for s, g in zip(S, gathered):
                L.check(s.lib.rmt_slab_extrapolate(s.h, g.data_ptr(), self._counts, cap),
                        "rmt_slab_extrapolate")
            self._mark(ev)
            # momentum (then the next step's geometry beside the projection), projection
            self._call("rmt_slab_momentum", dt)
            if k + 1 < nsteps and self.t + dt < t_end:
                geo = self._early_geometry()
            self._mark(ev)
            self._call("rmt_slab_project_rows", dt)
            sp = [s.a2a_splits() for s in S]
            comm.all_to_all([s.view("A") for s in S], [s.view("B") for s in S],
                            [x[0] for x in sp], [x[1] for x in sp])
            self._call("rmt_slab_project_cols")
            comm.all_to_all([s.view("B") for s in S], [s.view("A") for s in S],
                            [x[1] for x in sp], [x[0] for x in sp])
            self._call("rmt_slab_project_unrows")
            self._sub_mean(0)
            comm.halo(S, ("pc",), 2)
            self._call("rmt_slab_project_correct", dt)
            self._sub_mean(1)
            self._mark(ev)
            self._call("rmt_slab_finish")
            self._mark(ev)
            sc = self._scalars()
            self.t += dt
            self._record(sc, dt, m2)
            if ev:
                for k, name in enumerate(self.PHASES[:6]):
                    self._ms[name] += ev[k].elapsed_time(ev[k + 1])
                ms2 = (ctypes.c_double * 2)()
                L.check(L.lib().rmt_ctx_kernel_ms(self.ctx.h, ms2))
                self._ms["rk4_stage_kernels"] += ms2[0]
                self._ms["extrap_chain_kernel"] += ms2[1]
                self._nprof += 1
        self._call("rmt_slab_drop_geometry")

    def _early_geometry(self):
        """The next step's known plane (owned rows of phi after the fix-up), allgathered, and
        its extrapolation geometry on each slab's second stream beside the projection
        (rmt_sim_step's early geometry; RMT_SLAB_EARLY_GEO=0 turns it off)."""
        if not self._early_geo:
            return False
        self._call("rmt_slab_next_bits")
        self.comm.allgather_rows(self.slabs, "bits_next")
        self._call("rmt_slab_geometry")
        return True

    def _set_dev_dt(self, on):
        for s in self.slabs:
            L.check(s.lib.rmt_slab_set_device_dt(s.h, int(bool(on))), "rmt_slab_set_device_dt")
        if not on:
            self._dev_dt = False

    def _step_async(self, nsteps):
        """The step of step() with dt computed on the device (rmt_slab_next_dt: the host's
        expression on the allgathered max |u|^2), the rim allgathered at a fixed capacity
        (rmt_slab_rim_cap flags an overflow, raised at the next read-back) with the counts
        read on the device (rmt_slab_extrapolate_dev), and each step's dt and scalar blocks
        recorded in a device ring that the host reads every sync_every steps."""
        torch, comm, S, G = self.torch, self.comm, self.slabs, self.G
        self._set_dev_dt(True)
        if not self._dev_dt:
            gs = comm.allgather([s.view("scal") for s in S])[0]
            for s in S:
                L.check(s.lib.rmt_slab_next_dt(s.h, gs.data_ptr(), G, None), "rmt_slab_next_dt")
            self._dev_dt = True
        width = 2 + G * SC_N
        ring = torch.empty((self.sync_every, width), dtype=torch.float64,
                           device=S[0].view("scal").device)
        keep, slot = [], 0
        # each window of sync_every steps starts from a snapshot of the slabs' owned rows: a
        # rim that outgrows the fixed capacity (seen only at the window's read-back) sends the
        # window back to it and through the synchronous path, which moves the exact counts --
        # the same results the asynchronous path gives when the capacity holds
        snap, done = None, 0

        def snapshot():
            # one preallocated buffer per slab and field, reused by every window (copy_: no
            # allocation, and no second copy of the state alive per window)
            buf = getattr(self, "_snap_buf", None)
            if buf is None:
                buf = self._snap_buf = [{f: s.view(f)[s.r0 - s.lo:s.r1 - s.lo].clone()
                                         for f in _STATE} for s in S]
            else:
                for s, b in zip(S, buf):
                    for f in _STATE:
                        b[f].copy_(s.view(f)[s.r0 - s.lo:s.r1 - s.lo])
            return buf, self.t, len(self.records), done

        def restore(sn):
            own, t, nrec, d = sn
            for s, o in zip(S, own):
                for f in _STATE:
                    s.view(f)[s.r0 - s.lo:s.r1 - s.lo].copy_(o[f])
            self.t = t
            del self.records[nrec:]
            return d

        def flush():
            nonlocal slot, keep
            if not slot:
                return True
            rows = ring[:slot].cpu().numpy()
            slot, keep = 0, []
            over = [int(np.bitwise_or.reduce(r[2:].reshape(G, SC_N)[:, SC_FLAGS].astype(np.int64))) & 8
                    for r in rows]
            if any(over):
                need = max(float(r[2:].reshape(G, SC_N)[:, SC_COUNT].max()) for r in rows)
                self._rim_cap = max(self._rim_cap, _rim_capacity(need))
                return False
            for r in rows:
                sc = r[2:].reshape(G, SC_N)
                self.t += float(r[0])
                self._record(sc, float(r[0]), float(r[1]))
                self._rim_cap = max(self._rim_cap, _rim_capacity(sc[:, SC_COUNT].max()))
            return True

        def rerun():
            """back to the window's snapshot, the window's steps synchronously"""
            nonlocal snap, geo
            self._call("rmt_slab_drop_geometry")
            d0 = restore(snap)
            self.m2 = None
            self._call("rmt_slab_begin")
            self.m2 = float(self._scalars()[:, SC_M2].max())
            self._step_sync(done - d0, math.inf)
            self.reruns = getattr(self, "reruns", 0) + 1
            self._set_dev_dt(True)
            gs = comm.allgather([s.view("scal") for s in S])[0]
            for s in S:
                L.check(s.lib.rmt_slab_next_dt(s.h, gs.data_ptr(), G, None), "rmt_slab_next_dt")
            self._dev_dt = True   # the next step() need not repeat the dt allgather
            geo = False

        geo = False
        for k in range(nsteps):
            if slot == 0:
                snap = snapshot()
            h = comm.halo_start(S, ("u", "v", "p", "X1", "X2"), HALO)
            self._call("rmt_slab_advect_interior", 0.0)
            comm.halo_finish(h)
            self._call("rmt_slab_advect", 0.0)
            if not geo:   # else the plane was gathered with the early geometry
                comm.allgather_rows(S, "bits")
            geo = False
            self._call("rmt_slab_rim_pack")
            if self._rim_cap is None:   # once: the capacity from the first rim (host read)
                self._rim_cap = _rim_capacity(self._scalars()[:, SC_COUNT].max())
            # never more than the smallest slab owns (equal on every rank: the global splits)
            cap = min(self._rim_cap, self._min_owned)
            for s in S:
                L.check(s.lib.rmt_slab_rim_cap(s.h, cap), "rmt_slab_rim_cap")
            gs = comm.allgather([s.view("scal") for s in S])[0]
            rims = comm.allgather([s.view("rim").reshape(-1)[:max(cap, 1) * 3] for s in S])
            for s, g in zip(S, rims):
                L.check(s.lib.rmt_slab_extrapolate_dev(s.h, g.data_ptr(), gs.data_ptr(), cap),
                        "rmt_slab_extrapolate_dev")
            self._call("rmt_slab_momentum", 0.0)
            if k + 1 < nsteps:
                geo = self._early_geometry()
            self._call("rmt_slab_project_rows", 0.0)
            sp = [s.a2a_splits() for s in S]
            comm.all_to_all([s.view("A") for s in S], [s.view("B") for s in S],
                            [x[0] for x in sp], [x[1] for x in sp])
            self._call("rmt_slab_project_cols")
            comm.all_to_all([s.view("B") for s in S], [s.view("A") for s in S],
                            [x[1] for x in sp], [x[0] for x in sp])
            self._call("rmt_slab_project_unrows")
            self._sub_mean(0)
            comm.halo(S, ("pc",), 2)
            self._call("rmt_slab_project_correct", 0.0)
            self._sub_mean(1)
            self._call("rmt_slab_finish")
            gs2 = comm.allgather([s.view("scal") for s in S])[0]
            for k, s in enumerate(S):
                L.check(s.lib.rmt_slab_next_dt(s.h, gs2.data_ptr(), G,
                                               ring[slot].data_ptr() if k == 0 else None),
                        "rmt_slab_next_dt")
            keep += [gs, gs2]   # (librmt runs on torch's current stream: stream-ordered reuse)
            slot += 1
            done += 1
            if slot == self.sync_every and not flush():
                rerun()
        self._call("rmt_slab_drop_geometry")
        if not flush():
            rerun()
            self._call("rmt_slab_drop_geometry")

    def _sub_mean(self, which):
        roots = self.comm.allgather([s.view("scal")[SC_ROOT:SC_ROOT + 1] for s in self.slabs])
        for s, r in zip(self.slabs, roots):
            L.check(s.lib.rmt_slab_sub_mean(s.h, which, r.data_ptr()), "rmt_slab_sub_mean")

    def _record(self, sc, dt, m2):
        fl = int(np.bitwise_or.reduce(sc[:, SC_FLAGS].astype(np.int64)))
        if fl & 1:
            raise FloatingPointError("advect_reference_map: non-finite velocity (the "
                                     "simulation diverged)")
        if fl & 2:
            raise L.RMTError("slab step: a departure point left the halo rows")
        if fl & 4:
            who = [f"slab {k}: " + abort_detail(int(-sc[k, SC_FIT]))
                   for k in range(sc.shape[0]) if int(sc[k, SC_FLAGS]) & 4]
            raise L.RMTError("extrapolation sweep aborted (progress wait timed out; "
                             + "; ".join(who) + ")")
        d = sc[:, SC_DIAG:SC_DIAG + 10]
        sx, sy, cnt = (float(sum(d[:, k])) for k in (0, 1, 2))
        self.m2 = float(sc[:, SC_M2].max())
        self.records.append({
            "t": self.t, "dt": dt, "cx": sx / cnt if cnt > 0 else math.nan,
            "cy": sy / cnt if cnt > 0 else math.nan, "minJ": float(d[:, 3].min()),
            "maxJ": float(d[:, 4].max()), "umax": math.sqrt(m2),
            "fitted": int(sc[0, SC_FIT])})

    def diagnostics(self):
        keys = self.records[0].keys() if self.records else ()
        return {k: np.array([r[k] for r in self.records]) for k in keys}


_STATE = ("u", "v", "p", "X1", "X2")   # a step's inputs (owned rows; the halo is exchanged)


_ABORT_KINDS = ("?", "chain", "?", "?", "?", "?", "?", "relink order", "fallback sweep",
                "parallel combine")


def abort_detail(code):
    """The extrapolation's abort word (csrc/extrap.hpp EXA_*: tag | kind << 26 | part << 22 |
    id), as extrap_abort_detail (extrap.hip) words it: what stopped, in which chain part, at
    which fit (its ordinal within the part)."""
    if not code & (1 << 30):
        return "abort word %d" % code
    kind, part, ident = (code >> 26) & 15, (code >> 22) & 15, code & 0x3FFFFF
    name = _ABORT_KINDS[kind] if kind < len(_ABORT_KINDS) else "?"
    return f"{name} part {part}, fit ordinal {ident}"


def _rim_capacity(count):
    """Rim entries moved per slab by the asynchronous step: 1.5x the largest slab rim seen,
    rounded up to 4096 (a slab's rim grows by a few cells per step)."""
    return int(-(-int(1.5 * float(count) + 4096) // 4096) * 4096)


def soft_disc_in_lid_driven(N, comm, options=None):
    """Configs 2/4 physics (soft_disc_in_lid_driven.py:165-199), decomposed over comm.G
    slabs, from the driver's initial condition.  options: implementation switches of a
    context of the slabs' own (rmt_ctx_set_option), as simulation.Simulation takes them."""
    from .simulation import soft_disc_params, initial_disc_map
    kw = soft_disc_params(N)
    sim = DistributedSim(N, comm, options=options, **kw)
    X1, X2 = initial_disc_map(N, *kw["disc"], kw["layers"])
    z = np.zeros((N, N))
    sim.set_state(u=z, v=z, p=z, X1=X1, X2=X2)
    return sim


# ------------------------------------------------------------ MAC slabs (config 5) --
MS_N = 48            # RMT_MAC_SLAB_SCALARS
MS_FLAGS, MS_JMIN, MS_JMAX, MS_UMAX, MS_CEN, MS_COUNT, MS_ROOT, MS_FIT, MS_ANY = \
    0, 1, 2, 3, 4, 28, 36, 37, 38
MBUF = {"u": 0, "v": 1, "p": 2, "X1": 3, "X2": 4, "phi": 5, "bits": 6, "rim": 7, "A": 8,
        "B": 9, "scal": 10}


class MacSlab(Slab):
    """One rmt_mac_slab: cell rows [r0, r1) resident as [lo, hi); u faces like the cells,
    v faces rows lo .. hi (one extra top row).  Per-disc planes are named "X1:k"."""

    def __init__(self, ctx, params, G, rank, rsplits, csplits):
        self.lib = L.lib()
        rs = (ctypes.c_int * (G + 1))(*rsplits)
        cs = (ctypes.c_int * (G + 1))(*csplits)
        h = ctypes.c_void_p()
        L.check(self.lib.rmt_mac_slab_create(ctx.bind(), ctypes.byref(params), G, rank, rs, cs,
                                             ctypes.byref(h)), "rmt_mac_slab_create")
        self.h = h
        info = (ctypes.c_int * 8)()
        L.check(self.lib.rmt_mac_slab_info(h, info))
        self.r0, self.r1, self.lo, self.hi, self.c0, self.c1, self.W, _ = list(info)
        self.G, self.rank, self.splits, self.csplits = G, rank, list(rsplits), list(csplits)
        self.NY = self.NX = self.N = params.N
        self._views = {}

    def __del__(self):
        try:
            self.lib.rmt_mac_slab_destroy(self.h)
        except Exception:
            pass

    def top_extra(self, name):
        return 1 if name == "v" else 0

    def view(self, name):
        if name not in self._views:
            torch = F._torch()
            base, _, disc = name.partition(":")
            p = ctypes.c_void_p()
            L.check(self.lib.rmt_mac_slab_buffer(self.h, MBUF[base], int(disc or 0),
                                                 ctypes.byref(p)))
            N, nl, no = self.N, self.hi - self.lo, self.r1 - self.r0
            nc = self.c1 - self.c0
            shape = {"u": (nl, N + 1), "v": (nl + 1, N), "bits": (N, self.W),
                     "rim": (no * N, 3), "A": (no * N,), "B": (N * nc,),
                     "scal": (MS_N,)}.get(base, (nl, N))
            t = _wrap_device(torch, p.value, shape)
            if base == "bits":
                t = t.view(torch.int64)
            self._views[name] = t
        return self._views[name]


class MacDistributedSim:
    """The config-5 MAC step of rmt_mac_sim (mac.hip) decomposed into G row slabs.

    ``comm`` is a LocalComm or a TorchComm, as for DistributedSim.  Fields are bit-identical
    to ``mac.MacMultiDisc`` when every slab holds 2^m rows at a multiple of 2^m; the centroid
    diagnostics differ in summation order only.
    """

    def __init__(self, N, comm, specs, **physics):
        from .mac import mac_params
        torch = F._torch()
        self.torch, self.comm, self.N, self.G = torch, comm, N, comm.G
        self.specs = list(specs)
        self.K = len(self.specs)
        self.params, self.dt = mac_params(N, self.specs, **physics)
        self.dx = self.params.dx
        self.rsplits = even_splits(N, self.G, HALO + 1)
        self.csplits = even_splits(N, self.G, 2)
        self.ctx = F.ctx_for(N, N)
        self.slabs = [MacSlab(self.ctx, self.params, self.G, r, self.rsplits, self.csplits)
                      for r in comm.ranks]
        self.t = 0.0
        self.records = []
        self.diverged = False
        self._counts = (ctypes.c_longlong * self.G)()

    def set_state(self, u=None, v=None, p=None, maps=None):
        """Full host arrays (u (N, N+1), v (N+1, N), p (N, N), maps [(X1, X2, phi)] per disc)
        -> every slab's resident rows."""
        torch = self.torch
        items = [("u", u), ("v", v), ("p", p)]
        for k, m in enumerate(maps or ()):
            items += [(f"X1:{k}", m[0]), (f"X2:{k}", m[1]), (f"phi:{k}", m[2])]
        for name, arr in items:
            if arr is None:
                continue
            a = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float64))
            for s in self.slabs:
                dst = s.view(name)
                dst.copy_(a[s.lo:s.hi + s.top_extra(name)].to(dst.device))

    def gather(self, name):
        """The owned rows of every slab assembled into the full host array (v: N + 1 rows)."""
        torch = self.torch
        torch.cuda.synchronize()
        e = self.slabs[0].top_extra(name)
        last = self.G - 1
        def own(s):
            return s.view(name)[s.r0 - s.lo:s.r1 - s.lo + (e if s.rank == last else 0)]
        if isinstance(self.comm, LocalComm):
            return torch.cat([own(s) for s in self.slabs]).cpu().numpy()
        (s,) = self.slabs
        mine = own(s).contiguous()
        mx = max(self.rsplits[k + 1] - self.rsplits[k] for k in range(self.G)) + e
        pad = torch.zeros((mx, mine.shape[1]), dtype=torch.float64, device=mine.device)
        pad[:mine.shape[0]].copy_(mine)
        (g,) = self.comm.allgather([pad])
        g = g.reshape(self.G, mx, mine.shape[1]).cpu().numpy()
        return np.concatenate([g[k, :self.rsplits[k + 1] - self.rsplits[k] + (e if k == last else 0)]
                               for k in range(self.G)])

    def _call(self, fn, *args):
        for s in self.slabs:
            L.check(getattr(s.lib, fn)(s.h, *args), fn)

    def _scalars(self):
        g = self.comm.allgather([s.view("scal") for s in self.slabs])[0]
        return g.cpu().numpy().reshape(self.G, MS_N)

    PHASES = ("halo", "advect", "extrapolate", "predict", "projection", "correct")

    def set_profiling(self, on=True):
        """HIP events around each phase (summed over the local slabs); phase_times()."""
        self._prof = bool(on)
        self._ms = {k: 0.0 for k in self.PHASES}
        self._nprof = 0

    def phase_times(self):
        return {k: (v, self._nprof) for k, v in self._ms.items()}

    def _mark(self, ev):
        if getattr(self, "_prof", False):
            e = self.torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)

    def step(self, nsteps=1, t_end=math.inf):
        self.ctx.bind()
        comm, S, K = self.comm, self.slabs, self.K
        halo_planes = ["u", "v"] + [f"X{a}:{k}" for k in range(K) for a in (1, 2)]
        for _ in range(nsteps):
            if not (self.t < t_end) or self.diverged:
                break
            dt = self.dt
            if self.t + dt > t_end:
                dt = t_end - self.t
            ev = []
            self._mark(ev)
            comm.halo(S, halo_planes, HALO)
            self._mark(ev)
            self._call("rmt_mac_slab_advect", dt)
            self._mark(ev)
            for k in range(K):
                comm.allgather_rows(S, f"bits:{k}")
            self._call("rmt_mac_slab_rim_pack")
            sc = self._scalars()
            ident = 0
            for k in range(K):
                if not sc[:, MS_ANY + k].any():     # proven identity on every slab
                    self._call("rmt_mac_slab_extrapolate_identity", k)
                    ident += 1
                    continue
                counts = [int(c) for c in sc[:, MS_COUNT + k]]
                gathered, cap = comm.allgather_padded([s.view(f"rim:{k}") for s in S], counts, 3)
                for r, c in enumerate(counts):
                    self._counts[r] = c
                for s, g in zip(S, gathered):
                    L.check(s.lib.rmt_mac_slab_extrapolate(s.h, k, g.data_ptr(), self._counts,
                                                           cap), "rmt_mac_slab_extrapolate")
            self._mark(ev)
            self._call("rmt_mac_slab_predict", dt)
            self._mark(ev)
            roots = comm.allgather([s.view("scal")[MS_ROOT:MS_ROOT + 1] for s in S])
            for s, r in zip(S, roots):
                L.check(s.lib.rmt_mac_slab_project_rows(s.h, r.data_ptr()),
                        "rmt_mac_slab_project_rows")
            sp = [s.a2a_splits() for s in S]
            comm.all_to_all([s.view("A") for s in S], [s.view("B") for s in S],
                            [x[0] for x in sp], [x[1] for x in sp])
            self._call("rmt_mac_slab_project_cols")
            comm.all_to_all([s.view("B") for s in S], [s.view("A") for s in S],
                            [x[1] for x in sp], [x[0] for x in sp])
            self._call("rmt_mac_slab_project_unrows")
            self._mark(ev)
            comm.halo(S, ("p",), 1)
            self._call("rmt_mac_slab_correct", dt)
            self._mark(ev)
            sc = self._scalars()
            self.t += dt
            self._record(sc, dt)
            self.records[-1]["identity_discs"] = ident
            if ev:
                for k, name in enumerate(self.PHASES):
                    self._ms[name] += ev[k].elapsed_time(ev[k + 1])
                self._nprof += 1

    def _record(self, sc, dt):
        fl = int(np.bitwise_or.reduce(sc[:, MS_FLAGS].astype(np.int64)))
        if fl & 1:
            raise FloatingPointError("advect_reference_map: non-finite velocity (the "
                                     "simulation diverged)")
        if fl & 2:
            raise L.RMTError("MAC slab step: a departure point left the halo rows")
        if fl & 4:
            raise L.RMTError("extrapolation sweep aborted (progress wait timed out)")
        rec = {"t": self.t, "dt": dt, "minJ": float(sc[:, MS_JMIN].min()),
               "maxJ": float(sc[:, MS_JMAX].max()), "umax": float(sc[:, MS_UMAX].max()),
               "fitted": int(sc[:, MS_FIT].sum())}
        cen = sc[:, MS_CEN:MS_CEN + 3 * self.K].sum(axis=0)
        rec["cx"] = [cen[3 * k] / cen[3 * k + 2] if cen[3 * k + 2] > 0 else math.nan
                     for k in range(self.K)]
        rec["cy"] = [cen[3 * k + 1] / cen[3 * k + 2] if cen[3 * k + 2] > 0 else math.nan
                     for k in range(self.K)]
        # mac_multi_disc_lid.py:100-103: stop on non-finite u, J < 0, J > 20 or a lost disc
        lost = any(not cen[3 * k + 2] > 0 for k in range(self.K))
        rec["diverged"] = int(not math.isfinite(rec["umax"]) or rec["minJ"] < 0.0
                              or rec["maxJ"] > 20.0 or lost)
        self.diverged = bool(rec["diverged"])
        self.records.append(rec)

    def diagnostics(self):
        keys = self.records[0].keys() if self.records else ()
        return {k: np.array([r[k] for r in self.records]) for k in keys}


def mac_multi_disc_lid(N, comm, n_discs=3, seed=3, specs=None, **physics):
    """Config 5 (benchmarks/mac_multi_disc_lid.py:36-98) decomposed over comm.G slabs, from
    the driver's initial condition (same disc placement as mac.MacMultiDisc)."""
    from .mac import place_discs, initial_maps
    specs = list(specs) if specs is not None else place_discs(n_discs, seed)
    sim = MacDistributedSim(N, comm, specs, **physics)
    z = np.zeros
    sim.set_state(u=z((N, N + 1)), v=z((N + 1, N)), p=z((N, N)), maps=initial_maps(N, specs))
    return sim
