"""Tile transport between ranks (one process per GPU).

Backed by ``torch.distributed``: RCCL (backend "nccl") over xGMI on GPU,
gloo on CPU.  Collectives are issued from inside a taskpool task, i.e. with
the task's stream current: the collective waits for that stream's prior
work, and ``work.wait()`` makes the stream (not the host) wait for the
transfer, so communication overlaps the other streams' compute.

Patterns used by the algorithms (SURVEY.md §2.10 collective inventory):
* ``bcast``      -- panel diagonal tile to the owner column, panel piece
                    along a process row (direct fan-out; RCCL picks the
                    algorithm per message size);
* ``allgather``  -- panel pieces across a process column (in place);
* ``allreduce``  -- info / norm reductions.

Loopback rehearsal (``DPLASMA_LOOPBACK=1`` on a world-1 process group): the algorithms plan
their exchanges as if the rank's own tiles lived on another rank -- every tile edge that would
cross ranks on a real grid (and, for tile DAGs / tile programs, every operand edge) becomes a
send to and a receive from the rank itself.  On RCCL those are real ``ncclSend`` / ``ncclRecv``
pairs in one group (NCCL supports self-sends; only torch's Python front end refuses them,
``_check_not_self_rank``, which :func:`self_p2p` lifts for the duration of the call), so every
RCCL branch of the transport (grouped p2p batches, the urgent / bulk communicators, the
dataflow ``Transport`` of tile DAGs, all-to-all exchanges) executes on a one-GPU box with
results that must equal the exchange-free path.  gloo cannot connect a rank to itself: there
the self pairs are completed by a local copy (the CPU tests check the planning).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.distributed as dist


# ------------------------------------------------------------------ communication-order recorder
# Every rank issues its transfers from the same SPMD program: tasks are built in the same order on every
# rank (runtime/taskpool.py chains the communicating tasks in program order under any scheduler policy),
# so on every communicator each pair of ranks posts its messages in one order, and the batches of all
# communicators follow one global order of task labels -- the two conditions under which RCCL batches on
# several communicators (urgent / bulk / row / col, each on its own stream) cannot wait on each other in
# a cycle.  record() logs (label, communicator, op, peer, bytes) per call; check_order() verifies both
# conditions over every rank's log (tests/test_comm_order.py).
LABEL = ""            # the running task's name (set by the taskpool runner)
_GROUP_NAMES = {}
_REC = None


def name_group(group, name: str) -> None:
    if group is not None:
        _GROUP_NAMES[id(group)] = name


def _gname(group) -> str:
    return "world" if group is None else _GROUP_NAMES.get(id(group), f"g{id(group)}")


def record(on: bool = True):
    """Start (on) or stop recording this process's transfers; returns the log recorded so far."""
    global _REC
    log = _REC
    _REC = [] if on else None
    return log


def _rec_p2p(sends, recvs, group):
    if _REC is None:
        return
    g = _gname(group)
    batch = []
    for t, p in sends:
        batch.append(("send", int(p), _nbytes(t)))
    for t, p in recvs:
        batch.append(("recv", int(p), _nbytes(t)))
    _REC.append((LABEL, g, "p2p", batch))


def _rec_coll(kind, t, group):
    """t None: a collective whose per-rank sizes differ by design (all-to-all): only its kind is compared."""
    if _REC is not None:
        _REC.append((LABEL, _gname(group), kind, [("coll", -1, _nbytes(t) if t is not None else -1)]))


def check_order(logs: dict) -> None:
    """logs: rank -> record() log.  Raises AssertionError unless (1) on every communicator, the messages
    rank a sends to rank b and those b receives from a pair up in order (same sizes), (2) every member of a
    communicator issues the same sequence of collectives on it, and (3) the batches of all ranks follow one
    global order: merging every batch with the batches its messages pair with (the sender's DSEND(k) and the
    receiver's DRECV(k) are one transfer), the per-rank issue orders leave no cycle -- the condition under
    which no set of ranks can each wait, in issue order, for a batch that waits on another of them."""
    from collections import defaultdict
    sends, recvs, colls = defaultdict(list), defaultdict(list), defaultdict(dict)
    for r, log in logs.items():
        for bi, (label, g, kind, batch) in enumerate(log):
            for op, peer, nb in batch:
                if op == "send":
                    sends[(g, r, peer)].append((nb, (r, bi), label))
                elif op == "recv":
                    recvs[(g, peer, r)].append((nb, (r, bi), label))
                else:
                    colls[g].setdefault(r, []).append((kind, nb, (r, bi)))
    parent = {}

    def find(x):
        parent.setdefault(x, x)
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    def union(x, y):
        parent[find(x)] = find(y)
    for key in set(sends) | set(recvs):
        a, b = sends.get(key, []), recvs.get(key, [])
        for n in range(max(len(a), len(b))):
            if n >= len(a) or n >= len(b) or a[n][0] != b[n][0]:
                raise AssertionError(
                    f"communicator {key[0]}: rank {key[1]} -> {key[2]}: message {n} differs (sent "
                    f"{a[n][::2] if n < len(a) else None}, received {b[n][::2] if n < len(b) else None})")
            union(a[n][1], b[n][1])
    for g, per in colls.items():
        seqs = list(per.values())
        if any([x[:2] for x in sq] != [x[:2] for x in seqs[0]] for sq in seqs):
            raise AssertionError(f"communicator {g}: ranks issue different collective sequences")
        for i in range(len(seqs[0])):
            for sq in seqs[1:]:
                union(sq[i][2], seqs[0][i][2])
    succ, indeg, nodes = defaultdict(set), defaultdict(int), set()
    for r, log in logs.items():
        prev = None
        for bi in range(len(log)):
            c = find((r, bi))
            nodes.add(c)
            if prev is not None and prev != c and c not in succ[prev]:
                succ[prev].add(c)
                indeg[c] += 1
            if prev is not None and prev == c:
                raise AssertionError(f"rank {r}: batches {bi - 1} and {bi} pair with each other (a wait cycle)")
            prev = c
    ready = [n for n in nodes if indeg[n] == 0]
    seen = 0
    while ready:
        n = ready.pop()
        seen += 1
        for m in succ[n]:
            indeg[m] -= 1
            if indeg[m] == 0:
                ready.append(m)
    if seen != len(nodes):
        raise AssertionError("the ranks issue their batches in orders with no common global order "
                             f"({len(nodes) - seen} transfers on a cycle)")


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def loopback() -> bool:
    """True when the loopback rehearsal is on: DPLASMA_LOOPBACK=1 and a world-1 process group."""
    return (os.environ.get("DPLASMA_LOOPBACK", "0") == "1" and dist.is_available() and dist.is_initialized()
            and dist.get_world_size() == 1)


@contextlib.contextmanager
def self_p2p():
    """Let torch.distributed post sends / receives whose peer is this rank (loopback only)."""
    if not loopback():
        yield
        return
    import torch.distributed.distributed_c10d as c10d
    orig = c10d._check_not_self_rank
    c10d._check_not_self_rank = lambda *a, **k: None
    try:
        yield
    finally:
        c10d._check_not_self_rank = orig


def _split_self(sends, recvs):
    """gloo loopback: complete the self pairs (in order) with local copies; returns the rest."""
    me = dist.get_rank() if dist.is_initialized() else 0
    ss = [t for t, p in sends if p == me]
    rs = [t for t, p in recvs if p == me]
    if len(ss) != len(rs):
        raise RuntimeError(f"loopback: {len(ss)} self-sends but {len(rs)} self-receives in one batch")
    for a, b in zip(ss, rs):
        b.copy_(a.view(-1)[: b.numel()].view_as(b))
    return [(t, p) for t, p in sends if p != me], [(t, p) for t, p in recvs if p != me]


def bcast(t: torch.Tensor, src_global: int, group, world: bool = False) -> None:
    """Broadcast from global rank src_global over ``group`` (None: nothing to do -- unless ``world``,
    then over every rank)."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("bcast", _nbytes(t), group)
    if group is None and not world:
        return
    _rec_coll("bcast", t, group)
    if world and not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    w = dist.broadcast(t, src=src_global, group=group, async_op=True)
    w.wait()


def barrier_world() -> None:
    """A host-side barrier over every rank (the host returns once every rank has reached it)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    if _nccl():
        t = torch.zeros(1, device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t)
        torch.cuda.current_stream().synchronize()
    else:
        dist.barrier()


def _nccl() -> bool:
    return dist.get_backend() == "nccl"


def allgather_inplace(out: torch.Tensor, my_index: int, group) -> None:
    """out is [n_in_group, ...] contiguous; slot my_index already holds my contribution."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("allgather", _nbytes(out) - _nbytes(out[my_index]), group)
    if group is None:
        return
    _rec_coll("allgather", out, group)
    inp = out[my_index]
    if out.device.type == "cuda" and _nccl():
        w = dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1),
                                        group=group, async_op=True)
        w.wait()
    else:
        parts = list(out.unbind(0))
        mine = inp.clone()
        w = dist.all_gather(parts, mine, group=group, async_op=True)
        w.wait()


def allreduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> None:
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("allreduce", 2 * _nbytes(t), group)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    _rec_coll("allreduce", t, group)
    dist.all_reduce(t, op=op, group=group)


def p2p(sends=(), recvs=(), group=None) -> None:
    """Grouped point-to-point transfer: sends / recvs are lists of (tensor, global peer rank), on the
    communicator of ``group`` (None: the world's).

    RCCL: one grouped send/recv call (every pair on its own xGMI link); the current stream waits
    for the transfer.  gloo: CUDA tensors are staged through host memory (gloo moves host buffers)."""
    sends, recvs = list(sends), list(recvs)
    if not sends and not recvs:
        return
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        # critical link: per peer the larger direction (an xGMI link is full duplex: what I send to a peer and what
        # it sends me travel at the same time)
        out_b, in_b = {}, {}
        for t_, p_ in sends:
            out_b[p_] = out_b.get(p_, 0) + _nbytes(t_)
        for t_, p_ in recvs:
            in_b[p_] = in_b.get(p_, 0) + _nbytes(t_)
        crit = max(max(out_b.get(p_, 0), in_b.get(p_, 0)) for p_ in set(out_b) | set(in_b))
        return _BACKEND.sync("p2p", crit, group)
    _rec_p2p(sends, recvs, group)
    if _nccl():
        ops = [dist.P2POp(dist.isend, t, p, group=group) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=group) for t, p in recvs]
        with self_p2p():
            for w in dist.batch_isend_irecv(ops) or ():
                w.wait()
        return
    if loopback():
        sends, recvs = _split_self(sends, recvs)
    host_r = [(t, t.cpu() if t.device.type != "cpu" else t) for t, _ in recvs]
    works = [dist.isend(t.cpu() if t.device.type != "cpu" else t, p, group=group) for t, p in sends]
    works += [dist.irecv(h, p, group=group) for (_, h), (_, p) in zip(host_r, recvs)]
    for w in works:
        w.wait()
    for t, h in host_r:
        if h is not t:
            t.copy_(h)


class Pending:
    """An exchange in flight (``start_p2p``), completed by ``finish`` on the consumer's side.
    Device transfers (RCCL) are waited for per consumer stream; host ones (gloo) once."""
    __slots__ = ("works", "host_recvs", "keep", "device", "streams", "done", "meta")

    def __init__(self, works, host_recvs=(), keep=(), device=False, meta=None):
        self.works, self.host_recvs, self.keep = list(works), list(host_recvs), keep
        self.device, self.streams, self.done, self.meta = device, set(), False, meta


_BACKEND = None   # replaces the torch.distributed transport (tools/replay_potrf.py: modelled xGMI timing)


def set_backend(b) -> None:
    """Install a transport backend with ``start_p2p(sends, recvs, group, hint)`` / ``finish(p)`` and
    optionally ``sync(kind, critical_bytes, group)`` for the blocking collectives (None: torch.distributed)."""
    global _BACKEND
    _BACKEND = b


def start_p2p(sends=(), recvs=(), group=None, hint=None) -> Optional[Pending]:
    """Issue a grouped point-to-point exchange and return at once.

    sends / recvs: lists of (tensor, global peer rank); ``group``: the process group whose
    communicator carries it (each group has its own RCCL stream, so exchanges on different groups
    proceed concurrently -- over different xGMI links when their peers differ).  RCCL: the transfer
    waits for the current stream's prior work and runs on the group's stream; ``finish`` (issued
    later, under the consumer's stream) makes that stream -- not the host -- wait.  gloo: CUDA
    tensors are staged through host memory; ``finish`` waits on the host and unstages.
    ``hint`` describes the producer's work for a modelling backend; the real transports ignore it."""
    sends, recvs = list(sends), list(recvs)
    if not sends and not recvs:
        return None
    if _BACKEND is not None:
        return _BACKEND.start_p2p(sends, recvs, group, hint)
    _rec_p2p(sends, recvs, group)
    if _nccl() and any(t.device.type == "cuda" for t, _ in sends + recvs):
        ops = [dist.P2POp(dist.isend, t, p, group=group) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=group) for t, p in recvs]
        with self_p2p():
            return Pending(dist.batch_isend_irecv(ops) or (), device=True)
    if loopback():
        sends, recvs = _split_self(sends, recvs)
    host_s = [(t.cpu() if t.device.type != "cpu" else t, p) for t, p in sends]
    host_r = [(t, t.cpu() if t.device.type != "cpu" else t, p) for t, p in recvs]
    works = [dist.isend(h, p, group=group) for h, p in host_s]
    works += [dist.irecv(h, p, group=group) for _, h, p in host_r]
    return Pending(works, [(t, h) for t, h, _ in host_r if h is not t], keep=host_s)


def finish(p: Optional[Pending]) -> None:
    """Complete an exchange from ``start_p2p`` for the caller: RCCL -- the current stream waits for
    the transfer (once per stream); gloo -- the host waits and unstages (once).  None: no-op."""
    if p is None or p.done:
        return
    if p.device:
        sid = torch.cuda.current_stream().cuda_stream
        if sid in p.streams:
            return
        p.streams.add(sid)
        if _BACKEND is not None:
            _BACKEND.finish(p)
        else:
            for w in p.works:
                w.wait()
        return
    if _BACKEND is not None:
        _BACKEND.finish(p)
    else:
        for w in p.works:
            w.wait()
        for t, h in p.host_recvs:
            t.copy_(h)
    p.done = True


def exchange_add(t: torch.Tensor, peer: int, tmp: torch.Tensor) -> None:
    """t += (peer's t): symmetric pairwise sum through one send/recv pair (tmp: same size as t)."""
    p2p([(t, peer)], [(tmp[: t.numel()], peer)])
    t.add_(tmp[: t.numel()])


_TRI_IDX = {}


def _tri_index(n: int, ld: int, lower: bool, device) -> torch.Tensor:
    """Element offsets (column-major, leading dimension ld) of the lower / upper triangle of an n x n
    block, diagonal included -- n (n + 1) / 2 entries."""
    key = (n, ld, lower, str(device))
    t = _TRI_IDX.get(key)
    if t is None:
        r = torch.arange(n).view(-1, 1)
        c = torch.arange(n).view(1, -1)
        mask = (r >= c) if lower else (r <= c)
        off = (r + c * ld).expand(n, n)
        t = _TRI_IDX[key] = off.t()[mask.t()].contiguous().to(device)   # column by column
    return t


def bcast_tri(dst: torch.Tensor, dst_off: int, src: Optional[torch.Tensor], src_off: int, n: int, ld_src: int,
              ld_dst: int, lower: bool, root: int, group, pack: Optional[torch.Tensor] = None) -> None:
    """Broadcast only the lower / upper triangle of an n x n block (the reference's LOWER_TILE /
    UPPER_TILE arena shapes: half the bytes of the full tile).  The root reads its block from
    ``src[src_off]`` (leading dimension ld_src); every rank (root included) gets the triangle in
    ``dst[dst_off]`` (ld_dst); the rest of the destination block is not written."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("bcast", n * (n + 1) // 2 * dst.element_size(), group)
    if group is None:
        return
    nt = n * (n + 1) // 2
    buf = pack[:nt] if pack is not None else torch.empty(nt, dtype=dst.dtype, device=dst.device)
    if src is not None:
        buf.copy_(src.view(-1)[src_off + _tri_index(n, ld_src, lower, src.device)])
    bcast(buf, root, group)
    dst.view(-1)[dst_off + _tri_index(n, ld_dst, lower, dst.device)] = buf
