"""Execution context: the analogue of ``parsec_init``/``parsec_context_t``.

One process per GPU (``torch.distributed`` over RCCL on GPU, gloo on CPU).
The context owns

* the P x Q process grid (rank = prow*Q + pcol) and the row/column
  sub-communicators used for panel broadcasts (created once, like PaRSEC's
  remote-dependency engine communicator ``parsec_remote_dep_set_ctx``,
  ``src/scalapack_wrappers/dplasma_wrapper_parsec_init.c:112-114``);
* the device and its HIP streams: a high-priority ``panel`` stream for the
  critical-path tasks (POTRF/TRSM/panel broadcast), an ``update`` stream for
  the bulk trailing updates, and an ``aux`` stream;
* the native task runtime handle (``dplasma_amd.runtime``) and the per-call
  option registry (``dplasma_info``).

The taskpool lifecycle mirrors the reference: ``X_New`` builds a taskpool
(nothing runs), ``ctx.add_taskpool(tp)`` enqueues it, ``ctx.start()`` /
``ctx.wait()`` execute it (``src/dplasmaaux.h:98-102``).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.distributed as dist


def _default_grid(world: int):
    P = int(math.isqrt(world))
    while world % P:
        P -= 1
    return P, world // P


class Context:
    def __init__(self, nb_cores: Optional[int] = None, device=None, P: Optional[int] = None, Q: Optional[int] = None,
                 gpus: Optional[int] = None, verbose: int = 0):
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank() if self.distributed else 0
        self.world = dist.get_world_size() if self.distributed else 1
        self.verbose = verbose
        if P is None and Q is None:
            P, Q = _default_grid(self.world)
        elif P is None:
            P = self.world // Q
        elif Q is None:
            Q = self.world // P
        if P * Q != self.world:
            raise ValueError(f"grid {P}x{Q} does not match world size {self.world}")
        self.P, self.Q = P, Q
        self.myrow, self.mycol = self.rank // Q, self.rank % Q
        # device selection: one GPU per rank (LOCAL_RANK), or CPU
        if device is None:
            want_gpu = (gpus is None or gpus > 0) and torch.cuda.is_available()
            if want_gpu:
                nd = max(1, torch.cuda.device_count())
                lr = int(os.environ.get("LOCAL_RANK", self.rank % nd)) % nd
                device = torch.device("cuda", lr)
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            nd = max(1, torch.cuda.device_count())
            lr = int(os.environ.get("LOCAL_RANK", self.rank % nd)) % nd
            self.device = torch.device("cuda", lr)
        self.is_gpu = self.device.type == "cuda"
        self.nb_cores = nb_cores or int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        if self.is_gpu:
            torch.cuda.set_device(self.device)
            lo, hi = torch.cuda.Stream.priority_range()
            self.streams = {
                "panel": torch.cuda.Stream(device=self.device, priority=hi),
                "update": torch.cuda.Stream(device=self.device, priority=lo),
                "aux": torch.cuda.Stream(device=self.device, priority=lo),
            }
            ndiag = int(os.environ.get("DPLASMA_DIAG_CUS", "0"))
            if ndiag > 0:
                self._reserve_cus(ndiag)
        else:
            self.streams = {}
        self._groups_built = False
        # loopback rehearsal (parallel.comm.loopback): a world-1 group whose algorithms route their
        # would-be remote tile edges through RCCL sends / receives to the rank itself
        from .parallel import comm as _comm
        self.loopback = _comm.loopback()
        self.row_group = None
        self.col_group = None
        self.urgent_group = None
        self.bulk_groups = []
        self.row_ranks: List[int] = [self.myrow * Q + c for c in range(Q)]
        self.col_ranks: List[int] = [r * Q + self.mycol for r in range(P)]
        self._build_groups()
        if self.distributed and self.world > 1 and self.is_gpu and dist.get_backend() == "nccl":
            # bring the default communicator up on every rank now: the dataflow transport's grouped
            # send/recv (parallel.p2p) run on it and involve only the ranks with traffic, which must
            # never be the call that creates it
            t = torch.zeros(1, device=self.device)
            dist.all_reduce(t)
        self._queue = []
        # ready-queue policy of single-process taskpools (the reference's -o scheduler choice)
        self.scheduler = os.environ.get("DPLASMA_SCHEDULER", "") or None
        self.sched_seed = 0
        self.profiling = None  # utils.trace.Tracer when enabled
        self.dot_file = os.environ.get("DPLASMA_DOT") or None  # DOT dump of every compiled tile DAG
        if os.environ.get("DPLASMA_PROFILE"):
            from .utils.trace import Tracer
            self.profiling = Tracer(self)
        from .utils.info import Info
        self.info = Info()

    def _reserve_cus(self, ndiag: int):
        """Opt-in (DPLASMA_DIAG_CUS=n), POTRF only: a "diag" stream on CUs [0, n) for the
        latency-bound diagonal-tile factorisations and a "potrf_update" stream on the other CUs
        for POTRF's bulk trailing updates, so the tile kernel does not share SIMDs with the GEMM
        (HIP CU masks).  The shared "update" stream stays unmasked: the persistent LU / QR panel
        kernels size their grids for every CU and must not run on a masked stream."""
        import ctypes
        from .ops import _lib
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        nw = (ncu + 31) // 32
        diag, upd = [0] * nw, [0] * nw
        for c in range(ncu):
            if c < ndiag:
                diag[c // 32] |= 1 << (c % 32)
            else:
                upd[c // 32] |= 1 << (c % 32)
        lib = _lib.load()
        made = {}
        for name, m in (("diag", diag), ("potrf_update", upd)):
            arr = (ctypes.c_uint * nw)(*m)
            out = ctypes.c_void_p()
            rc = lib.dpl_stream_cumask(ctypes.cast(arr, ctypes.c_void_p), nw, ctypes.byref(out))
            _lib.check(rc, "stream_cumask")
            made[name] = torch.cuda.ExternalStream(out.value, device=self.device)
        self.streams.update(made)
        self._owned_streams = [s.cuda_stream for s in made.values()]

    @staticmethod
    def reserve_mask(ncu: int, reserve: int):
        """CU indices left to a bulk stream when ``reserve`` CUs are kept free for the critical path,
        spread evenly over the chip: 8 XCDs, and whichever way the HIP CU-mask bits map onto them
        (contiguous runs of ncu/8 or interleaved by index mod 8), every XCD keeps reserve/8 free CUs
        -- a workgroup of a critical-path kernel dealt to any XCD finds one."""
        per = ncu // 8
        r = max(0, min(per - 1, (reserve + 7) // 8))
        free = set()
        for x in range(8):
            for t in range(r):
                # column x*per + x + 8t: one per residue class mod 8 in each contiguous run
                free.add(x * per + (x + 8 * t) % per)
        return [c for c in range(ncu) if c not in free]

    def masked_stream(self, name: str, cus) -> str:
        """A HIP stream restricted to the CU indices ``cus`` (hipExtStreamCreateWithCUMask), registered
        as ``name`` and cached; destroyed by ``release``."""
        if name in self.streams:
            return name
        import ctypes
        from .ops import _lib
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        nw = (ncu + 31) // 32
        words = [0] * nw
        for c in cus:
            words[c // 32] |= 1 << (c % 32)
        arr = (ctypes.c_uint * nw)(*words)
        out = ctypes.c_void_p()
        lib = _lib.load()
        _lib.check(lib.dpl_stream_cumask(ctypes.cast(arr, ctypes.c_void_p), nw, ctypes.byref(out)), "stream_cumask")
        self.streams[name] = torch.cuda.ExternalStream(out.value, device=self.device)
        self._owned_streams = getattr(self, "_owned_streams", []) + [out.value]
        self._owned_names = getattr(self, "_owned_names", []) + [name]
        return name

    def bulk_stream(self, reserve: int):
        """A low-priority stream restricted to all CUs but ``reserve`` (see ``reserve_mask``); cached
        per reserve.  reserve <= 0 or no GPU: the plain ``update`` stream."""
        if reserve <= 0 or not self.is_gpu:
            return "update"
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        return self.masked_stream(f"bulk{reserve}", self.reserve_mask(ncu, reserve))

    def partition_streams(self, reserve: int):
        """(tile, chain, bulk) stream names for a CU partition: ``tile`` runs on the ``reserve`` CUs kept
        free by ``reserve_mask`` (the latency-bound diagonal-tile kernels alone on their CUs -- beside a
        GEMM's waves on the same SIMDs they run ~7x slower, profiles/r3_potrf_tile_cu_partition.txt),
        ``chain`` and ``bulk`` on the other CUs (the panel solves / look-ahead updates and the trailing
        update).  reserve <= 0 or no GPU: ("panel", "panel", "update")."""
        if reserve <= 0 or not self.is_gpu:
            return "panel", "panel", "update"
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        keep = self.reserve_mask(ncu, reserve)
        ks = set(keep)
        tile = self.masked_stream(f"tile{reserve}", [c for c in range(ncu) if c not in ks])
        chain = self.masked_stream(f"chain{reserve}", keep)
        return tile, chain, self.bulk_stream(reserve)

    def release(self):
        """Destroy the HIP streams this context created itself (CU-masked ones)."""
        owned = getattr(self, "_owned_streams", [])
        if owned:
            import gc

            from .ops import _lib
            # tensors the caching allocator handed out on these streams must go back to it while the streams
            # still exist: task pools hold reference cycles (closures), so without a collection here their
            # tensors were freed by a LATER garbage collection, onto destroyed streams -- a segfault inside an
            # unrelated test's import (GPU suite, round 6)
            gc.collect()
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()
            for name in ("diag", "potrf_update", *getattr(self, "_owned_names", [])):
                self.streams.pop(name, None)
            for s in owned:
                _lib.load().dpl_stream_destroy(s)
            self._owned_streams = []
            self._owned_names = []

    # ------------------------------------------------------------------ comms
    def _build_groups(self):
        if not self.distributed or (self.world == 1 and not self.loopback):
            return
        # every rank must create every group, in the same order.  On RCCL the panel traffic
        # (broadcasts / all-gathers of the factorisations' critical path) runs on high-priority
        # streams so its kernels are dispatched ahead of the bulk trailing-update GEMM workgroups.
        kw = {}
        if dist.get_backend() == "nccl":
            try:
                from torch.distributed import ProcessGroupNCCL
                opts = ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
            except Exception:  # pragma: no cover - older torch
                kw = {}
        rows, cols = [], []
        for r in range(self.P):
            ranks = [r * self.Q + c for c in range(self.Q)]
            rows.append(dist.new_group(ranks, **kw) if self.Q > 1 or self.loopback else None)
        for c in range(self.Q):
            ranks = [r * self.Q + c for r in range(self.P)]
            cols.append(dist.new_group(ranks, **kw) if self.P > 1 or self.loopback else None)
        self.row_group = rows[self.myrow]
        self.col_group = cols[self.mycol]
        # world-wide communicators of the dataflow tile transport (parallel.comm.start_p2p): one for
        # critical-path (look-ahead) traffic on high-priority RCCL streams and DPLASMA_BULK_GROUPS for
        # bulk traffic -- a communicator's operations are serialised on its stream, so bulk transfers
        # of consecutive panels (different roots, different xGMI links) only overlap on different ones
        nb = max(1, int(os.environ.get("DPLASMA_BULK_GROUPS", "2")))
        self.urgent_group = dist.new_group(list(range(self.world)), **kw)
        self.bulk_groups = [dist.new_group(list(range(self.world))) for _ in range(nb)]
        # names for the communication-order recorder (parallel.comm.record): the same on every rank
        from .parallel import comm as _comm
        for i, g in enumerate(rows):
            _comm.name_group(g, f"row{i}")
        for i, g in enumerate(cols):
            _comm.name_group(g, f"col{i}")
        _comm.name_group(self.urgent_group, "urgent")
        for i, g in enumerate(self.bulk_groups):
            _comm.name_group(g, f"bulk{i}")
        if dist.get_backend() == "nccl" and self.is_gpu:
            # create every communicator now, on every rank (a point-to-point batch that involves only
            # some ranks must never be the call that initialises one)
            t = torch.zeros(1, device=self.device)
            for g in [self.urgent_group, *self.bulk_groups, *[x for x in rows + cols if x is not None]]:
                dist.all_reduce(t, group=g)
        self._groups_built = True

    def barrier(self):
        if self.distributed and self.world > 1:
            if self.is_gpu:
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def sync(self):
        if self.is_gpu:
            torch.cuda.synchronize(self.device)

    def stream(self, name: str):
        return self.streams.get(name)

    def local(self) -> "Context":
        """A one-process view of this context (same device, streams and options, no communicators):
        the context of recursive sub-taskpools that run inside one task of this rank
        (reference: parsec_recursivecall, src/zpotrf_L.jdf:148-172)."""
        c = object.__new__(Context)
        c.__dict__.update(self.__dict__)
        c.distributed, c.rank, c.world = False, 0, 1
        c.loopback = False
        c.P, c.Q, c.myrow, c.mycol = 1, 1, 0, 0
        c.row_group = c.col_group = None
        c.urgent_group, c.bulk_groups = None, []
        c.row_ranks, c.col_ranks = [0], [0]
        c._queue = []
        return c

    # ------------------------------------------------------------------ taskpools
    def add_taskpool(self, tp):
        self._queue.append(tp)

    def start(self):
        for tp in self._queue:
            tp.run(self)

    def wait(self):
        for tp in self._queue:
            tp.complete(self)
        self._queue = []

    def __repr__(self):
        return f"Context(rank={self.rank}/{self.world}, grid={self.P}x{self.Q}, device={self.device})"


_DEFAULT: Optional[Context] = None


def init(nb_cores=None, device=None, P=None, Q=None, gpus=None, verbose=0) -> Context:
    """Create (or return) the default context -- ``parsec_init`` analogue."""
    global _DEFAULT
    _DEFAULT = Context(nb_cores=nb_cores, device=device, P=P, Q=Q, gpus=gpus, verbose=verbose)
    return _DEFAULT


def fini(ctx: Optional[Context] = None):
    global _DEFAULT
    c = ctx or _DEFAULT
    path = os.environ.get("DPLASMA_PROFILE")
    if c is not None and c.profiling is not None and path:
        c.profiling.dump(path if c.world == 1 else path)
    if c is not None:
        # cached LU exchange buffers (ops.lu_dist_ops): every rank of each process column unmaps them
        import sys
        ld = sys.modules.get("dplasma_amd.ops.lu_dist_ops")
        if ld is not None:
            ld.release_all()
        c.release()
    if ctx is None or ctx is _DEFAULT:
        _DEFAULT = None
