"""Cross-stream buffer hazards of the distributed LU task graph (models/lu.py _GetrfDev, P x Q with look-ahead).

On a GPU the tasks of one rank run on five streams -- PANEL / SWAPN / NEXT on "panel", the SWAPR chunks on "xch",
the REST chunks on "update", LEFT on "aux", LSEND on "lsend" -- and two tasks on different streams are ordered only by
a path of task edges.  This test runs the 2 x 4 program on the CPU (gloo, 8 ranks) with every kernel wrapper and
transfer instrumented: each task's reads and writes of the engine's scratch buffers (panel / U / staging / exchange
buffers, move lists, pivots -- everything but the matrix itself, whose tiles the DAG partitions) are recorded, and
every pair of tasks on different GPU streams that touch one buffer, one of them writing, must be ordered by the
graph.  Round 6 found two such races on the GPU (LSEND packing into the next panel's receive buffer; SWAPN and the
SWAPR chunks sharing a staging buffer); the negative control re-creates the second one and must be flagged.
"""
import pytest
import torch

from helpers import run_distributed

STREAM = (("PANEL(", "panel"), ("SWAPN(", "panel"), ("NEXT(", "panel"), ("LSEND(", "lsend"), ("SWAPR", "xch"),
          ("REST", "update"), ("LEFT(", "aux"), ("JOIN", "update"))


def _gpu_stream(name, streams=STREAM):
    for pre, s in streams:
        if name.startswith(pre):
            return s
    return "update"


def _worker(rank, world, N, NB, share):
    import os
    os.environ["DPLASMA_LU_PANEL"] = "gather"
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IPIV = dp.ptgpanel_ipiv_descriptor(ctx, A)
    tp = dp.getrf_ptgpanel_New(ctx, A, IPIV)
    st = tp._state
    assert st.xmode and st.lookahead
    if share == "staging":       # negative controls: the round-6 SWAPN / SWAPR race ...
        st.tmp_n = st.tmp
    elif share == "rsend":       # ... and LSEND packing into the receive buffer of the next panel
        assert st.lsend_task and st.rbuf_send is not None
        st.rbuf_send = [st.rbuf, st.rbuf]
    info, graph, acc = instrumented_run(ctx, tp, st, A)
    return info, graph, acc


def instrumented_run(ctx, tp, st, A):
    """Run taskpool tp with every scratch-buffer access of its tasks recorded: (info, graph, {task: (reads,
    writes)}), an access being (buffer name, first element, end element).  st: the engine object whose tensors are
    the scratch buffers (the matrix A is excluded)."""
    from dplasma_amd.ops import tile_ops as ops
    from dplasma_amd.parallel import comm
    # tracked scratch storages: every tensor the engine owns except the matrix
    names = {}

    def track(name, v):
        if isinstance(v, torch.Tensor):
            if v.numel():
                names.setdefault(v.untyped_storage().data_ptr(), name)
        elif isinstance(v, dict):
            for k, x in v.items():
                track(f"{name}.{k}", x)
        elif isinstance(v, (list, tuple)):
            for i, x in enumerate(v):
                track(f"{name}[{i}]", x)
    for k, v in st.__dict__.items():
        if k not in ("A", "ctx", "plan"):
            track(k, v)
    matrix = A.data.untyped_storage().data_ptr()
    names.pop(matrix, None)
    cur = [None]
    acc = {}    # task id -> (reads, writes)

    def note(ts, write):
        """ts: tensors, or (tensor, lo, hi) element ranges relative to the tensor's first element."""
        if cur[0] is None:
            return
        r, w = acc.setdefault(cur[0], (set(), set()))
        for x in ts:
            t, rng = (x[0], x[1:]) if isinstance(x, tuple) else (x, None)
            if isinstance(t, torch.Tensor) and t.numel():
                n = names.get(t.untyped_storage().data_ptr())
                if n:   # the element range touched (parity halves / chunks of one buffer do not conflict)
                    base = t.storage_offset()
                    if rng is None:
                        lo, hi = 0, sum((sz - 1) * sd for sz, sd in zip(t.shape, t.stride())) + 1
                    else:
                        lo, hi = rng
                    (w if write else r).add((n, base + lo, base + hi))

    import numpy as np

    def span(off, rows, cols, ld):
        off, rows, cols = (np.asarray(x, dtype=np.int64) for x in (off, rows, cols))
        if not off.size:
            return None
        return int(off.min()), int((off + (cols - 1) * ld + rows).max())

    def tile_rng(t, batch, which, ld):
        it = batch.items
        s_ = span(it["a_off"] if which == "a" else it["b_off"], it["m"], it["n"], ld)
        return [t] if s_ is None else [(t,) + s_]

    def gemm_rng(ta, tb, Ax, lda, B, ldb, C, ldc, batch):
        it, kp = batch.items, batch.kpairs
        if not len(it):
            return [], []
        rep = np.repeat(np.arange(len(it)), it["kt_cnt"])
        kk = kp[np.concatenate([np.arange(b, b + c) for b, c in zip(it["kt_beg"], it["kt_cnt"])])]
        m, n, k = it["m"][rep], it["n"][rep], kk["k"]
        ra = span(kk["a_off"], m, k, lda) if ta == 111 else span(kk["a_off"], k, m, lda)
        rb = span(kk["b_off"], k, n, ldb) if tb == 111 else span(kk["b_off"], n, k, ldb)
        rc = span(it["c_off"], it["m"], it["n"], ldc)
        return [(Ax,) + ra, (B,) + rb], [(C,) + rc]

    def wrap(mod, fname, rw):
        f = getattr(mod, fname)

        def g(*a, **k):
            rd, wr = rw(*a, **k)
            note(rd, False)
            note(wr, True)
            return f(*a, **k)
        setattr(mod, fname, g)
        return f

    def tens(x):
        if isinstance(x, torch.Tensor):
            return [x]
        if isinstance(x, (list, tuple)):
            return [y for y in x if isinstance(y, torch.Tensor)]
        return []
    saved = [
        (ops, "geadd", wrap(ops, "geadd", lambda part, tr, al, Ax, lda, be, B, ldb, batch, *r, **k:
                            (tile_rng(Ax, batch, "a", lda), tile_rng(B, batch, "b", ldb)))),
        (ops, "trsm", wrap(ops, "trsm", lambda s, u, t, d, al, Ax, lda, B, ldb, batch, *r, **k:
                           ([Ax], tile_rng(B, batch, "b", ldb)))),
        (ops, "gemm", wrap(ops, "gemm", lambda ta, tb, al, Ax, lda, B, ldb, be, C, ldc, batch, *r, **k:
                           gemm_rng(ta, tb, Ax, lda, B, ldb, C, ldc, batch))),
        (ops, "rows_move", wrap(ops, "rows_move", lambda g, Ax, ld, mb, r0, ro, co, nc, nb, idx, cnt, mx, buf, ldb,
                                *r, **k: (([Ax, idx, cnt], [(buf, 0, co.numel() * nb * ldb)]) if g
                                          else ([(buf, 0, co.numel() * nb * ldb), idx, cnt], [Ax])))),
        (ops, "rows_xcopy", wrap(ops, "rows_xcopy", lambda g, tmp, ldb, W, xo, cnt, mx, ptrs, nb, **k:
                                 (([(tmp, 0, W * ldb), xo, cnt], tens(ptrs)) if g
                                  else (tens(ptrs) + [xo, cnt], [(tmp, 0, W * ldb)])))),
        (ops, "piv_moves", wrap(ops, "piv_moves", lambda ip, kb, d, s_, c, *r, **k: ([ip], [d, s_, c]))),
        (ops, "rows_permute", wrap(ops, "rows_permute", lambda Ax, ld, mb, r0, ro, co, nc, nb, d, s_, c, *r, **k:
                                   ([d, s_, c], [Ax]))),
        (ops, "rows_xord", wrap(ops, "rows_xord", lambda md, ms, mc, *r, **k: ([md, ms, mc], [r[-2]]))),
        (comm, "p2p", wrap(comm, "p2p", lambda sends=(), recvs=(), group=None, **k:
                           ([t for t, _ in sends], [t for t, _ in recvs]))),
        (comm, "bcast", wrap(comm, "bcast", lambda t, *r, **k: ([], [t]))),
        (comm, "allreduce", wrap(comm, "allreduce", lambda t, *r, **k: ([], [t]))),
        (comm, "exchange_add", wrap(comm, "exchange_add", lambda t, peer, tmp: ([t], [t, tmp]))),
        (comm, "bcast_tri", wrap(comm, "bcast_tri", lambda dst, do, src, so, *r, **k: (tens(src), [dst]))),
        (ops, "sum_partials", wrap(ops, "sum_partials", lambda src, stride, S, L, dst: ([src], [(dst, 0, L)]))),
        (ops, "qr_panel", wrap(ops, "qr_panel", lambda P, ldp, M, nc, kf, V, ldv, Tm, ldt, ws, info, *r, **k:
                               ([P], [P, V, Tm, ws]))),
    ]
    pend = {}
    start0, finish0 = comm.start_p2p, comm.finish

    def start_p2p(sends=(), recvs=(), group=None, hint=None):
        # an asynchronous exchange writes its receive buffers (and reads its send buffers) from where it starts; the
        # tasks that finish it read them
        sd, rv = [t for t, _ in sends], [t for t, _ in recvs]
        note(sd, False)
        note(rv, True)
        h = start0(sends, recvs, group=group, hint=hint)
        if h is not None:
            pend[id(h)] = (sd, rv)
        return h

    def finish(h):
        if h is not None and id(h) in pend:   # a consumer observes the data (several consumers may finish one)
            sd, rv = pend[id(h)]
            note(sd + rv, False)
        return finish0(h)
    comm.start_p2p, comm.finish = start_p2p, finish
    saved += [(comm, "start_p2p", start0), (comm, "finish", finish0)]
    run0 = ops.PanelLU.run

    def run(self, ipiv, ws, cnt, info, base, *r, **k):
        note([], True)
        note([self.buf, ipiv, ws, cnt], True)
        return run0(self, ipiv, ws, cnt, info, base, *r, **k)
    ops.PanelLU.run = run
    copy0 = torch.Tensor.copy_

    def copy_(self, src, *r, **k):
        note([src], False)
        note([self], True)
        return copy0(self, src, *r, **k)
    torch.Tensor.copy_ = copy_
    for t in tp.tasks:
        def wrapped(fn=t.fn, tid=t.tid):
            cur[0] = tid
            try:
                fn()
            finally:
                cur[0] = None
        t.fn = wrapped
    try:
        info = tp.execute(ctx)
    finally:
        torch.Tensor.copy_ = copy0
        ops.PanelLU.run = run0
        for mod, fname, f in saved:
            setattr(mod, fname, f)
    graph = [(t.name, list(t.deps), t.stream) for t in tp.tasks]
    return info, graph, {k: (sorted(v[0]), sorted(v[1])) for k, v in acc.items()}


def _hazards(graph, acc, streams=STREAM):
    anc = []
    for _, deps, *_ in graph:
        a = set(deps)
        for d in deps:
            a |= anc[d]
        anc.append(a)
    by_buf = {}
    for tid, (rd, wr) in acc.items():
        for (b, lo, hi) in rd:
            by_buf.setdefault(b, []).append((tid, False, lo, hi))
        for (b, lo, hi) in wr:
            by_buf.setdefault(b, []).append((tid, True, lo, hi))
    out = set()
    for b, uses in by_buf.items():
        for i, (t1, w1, l1, h1) in enumerate(uses):
            for t2, w2, l2, h2 in uses[i + 1:]:
                if t1 == t2 or not (w1 or w2) or h1 <= l2 or h2 <= l1:
                    continue
                a, c = min(t1, t2), max(t1, t2)
                sa = _gpu_stream(graph[a][0], streams) if streams is not None else graph[a][2]
                sc = _gpu_stream(graph[c][0], streams) if streams is not None else graph[c][2]
                if sa == sc:
                    continue
                if a not in anc[c]:
                    out.add((b, graph[a][0], graph[c][0]))
    return sorted(out)


@pytest.mark.parametrize("share", ["none", "staging", "rsend"])
def test_lu_2x4_cross_stream_buffer_hazards(share):
    out = run_distributed(_worker, 8, 160, 16, share)
    found = []
    for r in range(8):
        info, graph, acc = out[r]
        assert info == 0
        found += [(r,) + h for h in _hazards(graph, acc)]
    if share == "staging":
        assert any(h[1] == "tmp" and {h[2][:5], h[3][:5]} == {"SWAPN", "SWAPR"} for h in found), found[:10]
    elif share == "rsend":
        assert any(h[1] == "rbuf" and {h[2][:5], h[3][:5]} == {"LSEND", "PANEL"} for h in found), found[:10]
    else:
        assert not found, found[:20]


P1_STREAMS = (("PANEL(", "panel"), ("NEXT(", "panel"), ("SWAP(", "update"), ("REST(", "update"), ("LEFTALL", "update"))


@pytest.mark.parametrize("M,N", [(256, 256), (320, 192)])
def test_lu_one_process_lookahead_hazards(M, N):
    """The one-process DGETRF defaults of round 6 (look-ahead PANEL / NEXT on the panel stream beside SWAP / REST, the
    deferred left pass at the end): no unordered cross-stream conflict on a scratch buffer."""
    import dplasma_amd as dp
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 32, 32, M, N)
    dp.plrnt(ctx, A, 11)
    IP = dp.ipiv_descriptor(ctx, A)
    tp = dp.getrf_1d_New(ctx, A, IP)
    st = tp._state
    assert st.lookahead and st.defer_left and len(st.pbufs) == 2
    info, graph, acc = instrumented_run(ctx, tp, st, A)
    assert info == 0
    assert any(g[0] == "LEFTALL" for g in graph)
    found = _hazards(graph, acc, P1_STREAMS)
    assert not found, found[:20]


LUQR_STREAMS = (("LU_PANEL(", "panel"), ("LU_NEXT(", "panel"), ("QR_PANELS(", "panel"), ("QR_NEXT(", "panel"),
                ("LU_SWAP(", "update"), ("LU_REST(", "update"), ("QR_REST(", "update"))


@pytest.mark.parametrize("crit,alpha", [(0, 1.0), (5, 50.0)])
def test_luqr_lookahead_hazards(monkeypatch, crit, alpha):
    """The hybrid LU-QR device path (one process, p = 1): LU and QR steps interleaved with look-ahead across them --
    no unordered cross-stream conflict on the LU engine's or the QR engine's scratch buffers."""
    import types

    import dplasma_amd as dp
    monkeypatch.setenv("DPLASMA_LUQR_FAST", "1")
    ctx = dp.init(device="cpu")
    N, NB, IB = 256, 32, 8
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3)
    TS = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N)
    TT = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N)
    IP = dp.qrf_ipiv_descriptor(ctx, A)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, 1, -1, -1, 1, -1, 0)
    tp = dp.getrf_qrf_New(ctx, tree, A, IP, TS, TT, crit, alpha, [0] * A.mt)
    assert tp.fast is not None and tp.fast.lookahead and tp.tasks
    st = types.SimpleNamespace(**{f"lu_{k}": v for k, v in tp.fast.__dict__.items() if k not in ("A", "ctx", "plan")},
                               **{f"qr_{k}": v for k, v in tp.qpf.__dict__.items() if k not in ("A", "ctx")})
    info, graph, acc = instrumented_run(ctx, tp, st, A)
    assert tp.complete(ctx) == 0
    kinds = {g[0].split("(")[0] for g in graph}
    assert {"LU_PANEL", "QR_PANELS"} <= kinds, kinds
    found = _hazards(graph, acc, LUQR_STREAMS)
    assert not found, found[:20]
