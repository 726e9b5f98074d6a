"""Dataflow tile transport: compile-time planned point-to-point exchanges.

The reference moves every tile edge of a PTG as soon as its producer finishes
(PaRSEC remote dependencies: ``src/zpotrf_L.jdf:109-114``, ``src/zgeqrf.jdf:84-121``).
Here the same effect is obtained without a runtime message engine: when a tile
program / tile DAG is compiled, every cross-rank tile edge is assigned to an
*exchange* (``Xfer``) that is

* issued at its **issue point** -- right after the compute level/stage that makes
  its data final (and after the receiver's last use of the slot it overwrites),
  not at the level that consumes it, so the transfer overlaps the compute of the
  levels in between;
* run only by the ranks that have traffic in it (grouped RCCL ``send``/``recv``
  with exactly the peers involved: ranks without traffic issue nothing);
* waited for by the compute stream only right before the first level that reads
  what it receives (``need``) and, on the sending side, before the first level
  that overwrites what it packed (``guard``).

GPU (RCCL): exchanges run on a dedicated communication stream.  The stream
waits for the compute stream's event at the issue point, packs the outgoing
tiles into a staging buffer (one batched copy launch per source), runs the
grouped p2p transfer, unpacks into the destination tiles, and records the
events the compute stream waits on.  Staging buffers are allocated once at
compile time (the communication stream serialises the exchanges, so one send and
one receive slab sized to the largest exchange suffice).

CPU (gloo) and the gloo-on-GPU rehearsal: sends are packed at the issue point
and posted asynchronously (``isend``/``irecv``); completion + unpack happen
lazily at the first level that needs the data (FIFO, and before any later
exchange packs a tile an in-flight one still has to write).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..constants import dplasmaNoTrans
from ..ops.batch import TileBatch
from ..utils import trace
from . import comm

# tile reference on this rank: (base index, element offset, ld, rows, cols, staging ld)
TileRef = Tuple[int, int, int, int, int, int]


def copy_tiles(A, lda, B, ldb, tb, to_b: bool):
    """Copy the tiles of a TileBatch (a_off in A, b_off in B) A -> B (to_b) or B -> A.

    Floating-point tiles use the batched copy kernel; integer tiles (pivot
    vectors) are tiny and copied with tensor views."""
    from ..ops import tile_ops as ops
    tb.finalize()
    if A.dtype.is_floating_point or A.dtype.is_complex:
        if to_b:
            ops.geadd(0, dplasmaNoTrans, 1.0, A, lda, 0.0, B, ldb, tb, copy=True)
            return
        sw = getattr(tb, "_swapped", None)
        if sw is None:
            sw = TileBatch()
            for it in tb.items:
                sw.add(int(it["b_off"]), int(it["m"]), int(it["n"]), b_off=int(it["a_off"]))
            sw.finalize()
            tb._swapped = sw
        ops.geadd(0, dplasmaNoTrans, 1.0, B, ldb, 0.0, A, lda, sw, copy=True)
        return
    for it in tb.items:
        m, n = int(it["m"]), int(it["n"])
        a = torch.as_strided(A, (m, n), (1, lda), int(it["a_off"]))
        b = torch.as_strided(B, (m, n), (1, ldb), int(it["b_off"]))
        (b if to_b else a).copy_(a if to_b else b)


class Xfer:
    """One exchange as seen by this rank: what it sends to / receives from each peer."""

    def __init__(self, xid: int, dtype, nbe: int, sends: Dict[int, List[TileRef]], recvs: Dict[int, List[TileRef]],
                 label: str = "", recv_into: Optional[Tuple[int, int]] = None):
        """recv_into = (base index, element offset): the received tiles are laid out exactly like the
        staging slab (per peer in ``recvs`` order, nbe apart, ld = staging ld) starting there, so
        they are received in place and there is no unpack."""
        self.xid, self.dtype, self.nbe, self.label = xid, dtype, nbe, label
        self.recv_into = recv_into
        self.send_peers = sorted(p for p, v in sends.items() if v)
        self.recv_peers = sorted(p for p, v in recvs.items() if v)
        self.send_seg, self.recv_seg = {}, {}
        self.pack: Dict[tuple, TileBatch] = {}
        self.unpack: Dict[tuple, TileBatch] = {}
        self.packs_set, self.unpacks_set = set(), set()
        pos = 0
        for p in self.send_peers:
            p0 = pos
            for (b, off, ld, r, c, sld) in sends[p]:
                self.pack.setdefault((b, ld, sld), TileBatch()).add(off, r, c, b_off=pos * nbe)
                self.packs_set.add((b, off))
                pos += 1
            self.send_seg[p] = (p0 * nbe, (pos - p0) * nbe)
        self.nsend = pos
        pos = 0
        for p in self.recv_peers:
            p0 = pos
            for (b, off, ld, r, c, sld) in recvs[p]:
                # staging -> tile: a = staging (ld sld), b = destination tile
                if recv_into is None:
                    self.unpack.setdefault((b, ld, sld), TileBatch()).add(pos * nbe, r, c, b_off=off)
                self.unpacks_set.add((b, off))
                pos += 1
            self.recv_seg[p] = (p0 * nbe, (pos - p0) * nbe)
        self.nrecv = pos
        for tb in list(self.pack.values()) + list(self.unpack.values()):
            tb.finalize()

    @property
    def active(self) -> bool:
        return bool(self.send_peers or self.recv_peers)

    def bytes_sent(self) -> int:
        return self.nsend * self.nbe * torch.empty(0, dtype=self.dtype).element_size()

    def do_pack(self, bases, sbuf):
        for (b, ld, sld), tb in self.pack.items():
            copy_tiles(bases[b], ld, sbuf, sld, tb, to_b=True)

    def recv_target(self, bases, rbuf):
        """Where the transfer lands: the destination slab itself (recv_into) or the staging slab."""
        if self.recv_into is None or self.nrecv == 0:
            return rbuf
        b, o = self.recv_into
        return bases[b][o:o + max(1, self.nrecv * self.nbe)]

    def do_unpack(self, rbuf, bases):
        if self.nrecv == 0:
            return
        if self.recv_into is not None:
            tgt = self.recv_target(bases, None)
            if rbuf.data_ptr() != tgt.data_ptr():
                tgt[: self.nrecv * self.nbe].copy_(rbuf[: self.nrecv * self.nbe])
            return
        for (b, ld, sld), tb in self.unpack.items():
            copy_tiles(rbuf, sld, bases[b], ld, tb, to_b=True)

    def p2p_ops(self, sbuf, rbuf):
        ops = []
        for p in self.send_peers:
            o, n = self.send_seg[p]
            ops.append(dist.P2POp(dist.isend, sbuf[o:o + n], p, tag=self.xid))
        for p in self.recv_peers:
            o, n = self.recv_seg[p]
            ops.append(dist.P2POp(dist.irecv, rbuf[o:o + n], p, tag=self.xid))
        return ops


class Transport:
    """The exchanges of one compiled program and when they run (see module docstring).

    ``add(xfer, point, need, guard)``: issue after compute level ``point`` (-1: at the start),
    the compute stream waits for completion before level ``need`` (None: at the end) and for
    the pack before level ``guard`` (None: never)."""

    def __init__(self, ctx, name: str, bases_fn: Callable[[], Sequence[torch.Tensor]]):
        self.ctx, self.name = ctx, name
        self.bases_fn = bases_fn
        self.at_point: Dict[int, List[Xfer]] = defaultdict(list)
        self.need_at: Dict[int, List[int]] = defaultdict(list)
        self.guard_at: Dict[int, List[int]] = defaultdict(list)
        self.xfers: List[Xfer] = []
        self.gpu_async = bool(ctx.is_gpu and dist.is_initialized() and dist.get_backend() == "nccl")
        self.stats = {"xfers": 0, "sends": 0, "recvs": 0, "bytes_sent": 0, "peers": set()}
        self.n_global = 0   # exchanges of the whole program (every rank); this rank runs len(self)
        self._sbuf: Dict[object, torch.Tensor] = {}
        self._rbuf: Dict[object, torch.Tensor] = {}
        self._finalized = False

    def add(self, x: Xfer, point: int, need: Optional[int], guard: Optional[int]):
        if not x.active:
            return
        if need is not None and need <= point:
            raise ValueError(f"{self.name}: exchange {x.label} needed at {need} but issued after {point}")
        self.xfers.append(x)
        self.at_point[point].append(x)
        if need is not None:
            self.need_at[need].append(x.xid)
        if guard is not None and self.gpu_async:
            self.guard_at[guard].append(x.xid)

    def __len__(self):
        return len(self.xfers)

    def finalize(self):
        """Allocate the staging slabs (GPU: one send + one receive slab per dtype, reused)."""
        if self._finalized:
            return self
        for pts in self.at_point.values():
            pts.sort(key=lambda x: x.xid)
        if self.gpu_async:
            dev = self.ctx.device
            ms, mr = defaultdict(int), defaultdict(int)
            for x in self.xfers:
                ms[x.dtype] = max(ms[x.dtype], x.nsend * x.nbe)
                mr[x.dtype] = max(mr[x.dtype], x.nrecv * x.nbe)
            for dt in set(ms) | set(mr):
                self._sbuf[dt] = torch.empty(max(1, ms[dt]), dtype=dt, device=dev)
                self._rbuf[dt] = torch.empty(max(1, mr[dt]), dtype=dt, device=dev)
            self.comm_stream = self.ctx.streams.get("comm") if hasattr(self.ctx, "streams") else None
            if self.comm_stream is None:
                lo, hi = torch.cuda.Stream.priority_range()
                self.comm_stream = torch.cuda.Stream(device=dev, priority=hi)
                self.ctx.streams["comm"] = self.comm_stream
        self._finalized = True
        return self

    # ------------------------------------------------------------------ run protocol
    def start(self, stream=None):
        """Beginning of a run: exchanges whose data is final before the first level."""
        self.finalize()
        self._done, self._packed = {}, {}
        self._inflight: List[tuple] = []
        self._bases = list(self.bases_fn())
        self.after(-1, stream)

    def before(self, level: int, stream=None):
        if self.gpu_async:
            for xid in self.need_at.get(level, ()):
                stream.wait_event(self._done[xid])
            for xid in self.guard_at.get(level, ()):
                stream.wait_event(self._packed[xid])
            return
        want = self.need_at.get(level)
        if want:
            self._complete(set(want))

    def after(self, level: int, stream=None):
        xs = self.at_point.get(level)
        if not xs:
            return
        if self.gpu_async:
            self._issue_gpu(xs, stream)
        else:
            for x in xs:
                self._post_cpu(x)

    def finish(self, stream=None):
        if self.gpu_async:
            if self.xfers:
                ev = torch.cuda.Event()
                ev.record(self.comm_stream)
                stream.wait_event(ev)
            return
        if self._inflight:
            self._complete({self._inflight[-1][0].xid})

    # ------------------------------------------------------------------ GPU (RCCL)
    def _issue_gpu(self, xs, stream):
        cs = self.comm_stream
        ev = torch.cuda.Event()
        ev.record(stream)
        cs.wait_event(ev)
        with torch.cuda.stream(cs):
            for x in xs:
                with trace.span(self.ctx, f"{self.name}:xfer", "comm", cs,
                                {"xid": x.xid, "send": x.nsend, "recv": x.nrecv, "peers": len(x.send_peers)}):
                    sb, rb = self._sbuf[x.dtype], self._rbuf[x.dtype]
                    x.do_pack(self._bases, sb)
                    pe = torch.cuda.Event()
                    pe.record(cs)
                    self._packed[x.xid] = pe
                    rt = x.recv_target(self._bases, rb)
                    ops_ = x.p2p_ops(sb, rt)
                    comm._rec_p2p([(o.tensor, o.peer) for o in ops_ if o.op is dist.isend],
                                  [(o.tensor, o.peer) for o in ops_ if o.op is dist.irecv], None)
                    with comm.self_p2p():
                        for w in dist.batch_isend_irecv(ops_) or ():
                            w.wait()
                    x.do_unpack(rt, self._bases)
                    de = torch.cuda.Event()
                    de.record(cs)
                    self._done[x.xid] = de
                self._count(x)

    # ------------------------------------------------------------------ CPU / gloo
    def _post_cpu(self, x: Xfer):
        # an in-flight exchange that still has to write a tile this one packs completes first
        hit = {y.xid for (y, _, _) in self._inflight if y.unpacks_set & x.packs_set}
        if hit:
            self._complete(hit)
        dev = self._bases[0].device if self._bases else torch.device("cpu")
        with trace.span(self.ctx, f"{self.name}:post", "comm", args={"xid": x.xid}, gpu=False):
            sb = torch.empty(max(1, x.nsend * x.nbe), dtype=x.dtype, device=dev)
            x.do_pack(self._bases, sb)
            if sb.device.type != "cpu":  # gloo moves host memory
                sb = sb.cpu()
            rb = torch.empty(max(1, x.nrecv * x.nbe), dtype=x.dtype)
            if x.recv_into is not None and dev.type == "cpu":
                rb = x.recv_target(self._bases, rb)   # receive in place
            p2p = x.p2p_ops(sb, rb)
            comm._rec_p2p([(o.tensor, o.peer) for o in p2p if o.op is dist.isend],
                          [(o.tensor, o.peer) for o in p2p if o.op is dist.irecv], None)
            if comm.loopback():   # gloo cannot reach the rank itself: self pairs become local copies
                comm._split_self([(o.tensor, o.peer) for o in p2p if o.op is dist.isend],
                                 [(o.tensor, o.peer) for o in p2p if o.op is dist.irecv])
                me = dist.get_rank()
                p2p = [o for o in p2p if o.peer != me]
            works = [dist.isend(op.tensor, op.peer, tag=x.xid) if op.op is dist.isend
                     else dist.irecv(op.tensor, op.peer, tag=x.xid) for op in p2p]
        self._inflight.append((x, works, (sb, rb)))
        self._count(x)

    def _complete(self, xids):
        """Complete (wait + unpack) the in-flight exchanges in posting order, up to the last of xids."""
        last = -1
        for i, (y, _, _) in enumerate(self._inflight):
            if y.xid in xids:
                last = i
        for _ in range(last + 1):
            x, works, (sb, rb) = self._inflight.pop(0)
            with trace.span(self.ctx, f"{self.name}:wait", "comm", args={"xid": x.xid}, gpu=False):
                for w in works:
                    w.wait()
                dev = self._bases[0].device if self._bases else torch.device("cpu")
                x.do_unpack(rb.to(dev) if dev.type != "cpu" else rb, self._bases)

    def _count(self, x: Xfer):
        self.stats["xfers"] += 1
        self.stats["sends"] += len(x.send_peers)
        self.stats["recvs"] += len(x.recv_peers)
        self.stats["bytes_sent"] += x.bytes_sent()
        self.stats["peers"].update(x.send_peers)
        self.stats["peers"].update(x.recv_peers)


def first_after(tab_keys: np.ndarray, tab_levels: np.ndarray, q_keys: np.ndarray, q_levels: np.ndarray,
                nlev: int) -> np.ndarray:
    """For each query (key, p): the smallest table level > p with the same key, or -1."""
    q_keys = np.asarray(q_keys, dtype=np.int64)
    if len(q_keys) == 0:
        return np.zeros(0, dtype=np.int64)
    if len(tab_keys) == 0:
        return np.full(len(q_keys), -1, dtype=np.int64)
    uk = np.unique(np.concatenate([np.asarray(tab_keys, dtype=np.int64), q_keys]))
    S = np.int64(nlev + 2)
    code_t = np.sort(np.searchsorted(uk, tab_keys).astype(np.int64) * S + (np.asarray(tab_levels) + 1))
    qi = np.searchsorted(uk, q_keys).astype(np.int64)
    code_q = qi * S + (np.asarray(q_levels, dtype=np.int64) + 1)
    idx = np.searchsorted(code_t, code_q, side="right")
    out = np.full(len(q_keys), -1, dtype=np.int64)
    ok = idx < len(code_t)
    hit = np.zeros(len(q_keys), dtype=bool)
    hit[ok] = (code_t[idx[ok]] // S) == qi[ok]
    out[hit] = code_t[idx[hit]] % S - 1
    return out
