"""Reference-style testing driver: ``python -m dplasma_amd.testing <prec><op> [flags]``.

Mirrors the ``tests/testing_z*.c`` programs and their common CLI
(``tests/common.c:171-259``): -N/-M/-K, -t/--MB, -T/--NB,
-i/--IB, -P/-Q, -x/--check, --seed, --mtx, --nruns, --qr_a/--qr_p/--treel/--treeh,
-d/--domino, -r/--tsrr, -v, --dot.  Each run prints the reference's result line

    [****] TIME(s)      t : dpotrf PxQxg=   P Q g NB=  nb N=    n :      X gflops - ENQ&PROG&DEST e p d

and, with -x, the check outcome ("Solution is CORRECT" / "SUSPICIOUS") using
the reference's residual tests (``src/dplasma_zcheck.c``, ``tests/testing_zgeqrf.c:221-303``).
Multi-process: launch with ``torch.distributed.run``; the grid is P x (world/P).
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch

PRECS = {"s": torch.float32, "d": torch.float64, "c": torch.complex64, "z": torch.complex128}
EPS = {"s": 5.96e-08, "d": 1.11e-16, "c": 5.96e-08, "z": 1.11e-16}


def _parse(argv):
    ap = argparse.ArgumentParser(prog="python -m dplasma_amd.testing", add_help=True)
    ap.add_argument("op", help="e.g. dpotrf, zgemm, dgeqrf_hqr, sgetrf_incpiv")
    ap.add_argument("-N", type=int, required=True)
    ap.add_argument("-M", type=int, default=0)
    ap.add_argument("-K", "--NRHS", type=int, default=0, dest="K")
    ap.add_argument("-t", "--MB", type=int, default=0, dest="MB")
    ap.add_argument("-T", "--NB", type=int, default=0, dest="NB")
    ap.add_argument("-i", "--IB", type=int, default=0, dest="IB")
    ap.add_argument("-P", "-p", "--grid-rows", type=int, default=0, dest="P")
    ap.add_argument("-Q", "-q", "--grid-cols", type=int, default=0, dest="Q")
    ap.add_argument("-x", "--check", action="store_true")
    ap.add_argument("-X", "--check_inv", action="store_true")
    ap.add_argument("--seed", type=int, default=3872)
    ap.add_argument("--mtx", type=int, default=0)
    ap.add_argument("--nruns", type=int, default=1)
    ap.add_argument("--qr_a", type=int, default=-1)
    ap.add_argument("--qr_p", type=int, default=-1)
    ap.add_argument("--treel", type=int, default=1)
    ap.add_argument("--treeh", type=int, default=-1, help="high-level tree (-1: flat, fibonacci when nt < mt/2)")
    ap.add_argument("-d", "--domino", type=int, nargs="?", const=1, default=-1,
                    help="domino coupling of the two trees (-1: on when nt < mt/2, as the reference)")
    ap.add_argument("-r", "--tsrr", action="store_true")
    ap.add_argument("-a", "--alpha", type=float, default=1.0)
    ap.add_argument("-u", "--uplo", default="L")
    ap.add_argument("-v", "--verbose", type=int, nargs="?", const=1, default=0)
    ap.add_argument("-g", "--gpus", type=int, default=-1, help="0: CPU only; default: GPU when present")
    ap.add_argument("--dot", default=None, help="write the DAG of DAG-based ops to this DOT file")
    ap.add_argument("--criteria", type=int, default=0, help="LU-QR criterion (include/dplasma/lu_qr.h)")
    ap.add_argument("--sim", action="store_true",
                    help="print the simulation date (critical path with the reference SIMCOST task costs) of "
                         "tile-DAG algorithms, as PaRSEC simulation builds do")
    ap.add_argument("--trace", default=None, help="write a Chrome trace (all ranks) of the timed runs to this file")
    # remaining flags of tests/common.c:171-259
    ap.add_argument("-s", "--kp", "--SMB", type=int, default=1, dest="kp", help="k-cyclic repetition over rows")
    ap.add_argument("-S", "--kq", "--SNB", type=int, default=1, dest="kq", help="k-cyclic repetition over cols")
    ap.add_argument("-A", "--LDA", type=int, default=0, dest="LDA", help="LAPACK storage with this local lld")
    ap.add_argument("-B", "--LDB", type=int, default=0, dest="LDB")
    ap.add_argument("-C", "--LDC", type=int, default=0, dest="LDC")
    ap.add_argument("-b", "--sync", action="store_true", help="synchronise (barrier) around every phase")
    ap.add_argument("-y", "--butlvl", type=int, default=0, help="butterfly level (hebut/gebut)")
    ap.add_argument("-z", "--HNB", "--HMB", type=int, default=0, dest="HNB",
                    help="recursive sub-tile size hint (dplasma_z*_setrecursive)")
    ap.add_argument("-c", "--cores", type=int, default=0, help="host worker threads (CPU path)")
    ap.add_argument("-m", "--thread_multi", action="store_true", help="accepted for compatibility")
    ap.add_argument("--ptg-to-dtd", "--ptg_to_dtd", action="store_true", dest="ptg_to_dtd",
                    help="re-execute every tile-DAG algorithm through the DTD front end (the reference's "
                         "--mca mca_pins ptg_to_dtd)")
    ap.add_argument("-o", "--scheduler", default="", help="ready-queue policy of the task issue order "
                    "(LFQ/LTQ/AP/LHQ/SPQ/PBQ: priority first, IP: inverse priority, GD: FIFO, LL: LIFO, RND: random; "
                    "default: program order); multi-process runs issue in program order")
    return ap.parse_args(argv)


class Harness:
    def __init__(self, a):
        self.a = a
        world = int(os.environ.get("WORLD_SIZE", "1"))
        import torch.distributed as dist
        if world > 1:
            # P x Q stream programs (LU / QR / Cholesky look-ahead) keep panel, update, exchange and side streams plus
            # one stream per communicator busy at once: one hardware queue each, or HIP's default of 4 per process
            # serialises them (2 x 4 LU rank replay: 32.5 % with 4 queues, 40.2 % with 16 -- profiles/r6_lu_config5.txt).
            # Must be set before HIP starts (torch.cuda.is_available() below starts it).
            os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
        use_gpu = torch.cuda.is_available() and a.gpus != 0
        if world > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if use_gpu:
                local = int(os.environ.get("LOCAL_RANK", "0"))
                torch.cuda.set_device(local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
        import dplasma_amd as dp
        self.dp = dp
        if a.ptg_to_dtd:
            from .runtime import dag as _dag
            _dag.PTG_TO_DTD[0] = True
        P = a.P or None
        if a.cores > 0:
            torch.set_num_threads(a.cores)
        self.ctx = dp.init(P=P, device=None if use_gpu else "cpu", nb_cores=a.cores or None)
        if a.scheduler:
            from .runtime.taskpool import policy_code
            policy_code(a.scheduler)   # unknown names fail here
            self.ctx.scheduler = a.scheduler
            if a.verbose:
                print(f"#+++++ scheduler {a.scheduler}: native ready-queue issue order", flush=True)
        self.prec = a.op[0]
        if self.prec not in PRECS:
            raise SystemExit(f"operation must start with a precision letter s/d/c/z: {a.op}")
        self.name = a.op[1:]
        self.dt = PRECS[self.prec]
        self.ok = True
        self.mats = []   # operands made by mat(): restored before every run after the first
        if a.dot:
            dp.dot_start(self.ctx, a.dot)
        if a.trace:
            dp.profiling_start(self.ctx)

    # ------------------------------------------------------------ helpers
    def mat(self, m, n, mb=None, nb=None, name="A"):
        a = self.a
        mb = mb or a.MB or a.NB or 180
        nb = nb or a.NB or mb
        lld = {"A": a.LDA, "B": a.LDB, "C": a.LDC}.get(name, 0)
        kw = {"kp": a.kp, "kq": a.kq}
        if lld:
            kw.update(storage=self.dp.STORAGE_LAPACK, lld=lld)
        M = self.dp.block_cyclic(self.ctx, self.dt, mb, nb, m, n, name=name, **kw)
        self.mats.append(M)
        return M

    def report(self, opname, t, flops, t_enq=0.0, t_dest=0.0):
        ctx = self.ctx
        if ctx.rank == 0:
            g = 1 if ctx.is_gpu else 0
            print(f"[****] TIME(s) {t:12.5f} : {self.prec}{opname}\tPxQxg= {ctx.P:3d} {ctx.Q:<3d} {g} "
                  f"NB= {self.a.NB or self.a.MB or 180:4d} N= {self.a.N:7d} : {flops / t / 1e9 if t > 0 else 0:14f} "
                  f"gflops - ENQ&PROG&DEST {t_enq:12.5f} : {t:12.5f} : {t_dest:12.5f}", flush=True)

    def run_tp(self, opname, build):
        """build() -> taskpool; times ENQ (build), PROG (run+complete), DEST; returns (taskpool result)."""
        ctx = self.ctx
        res = None
        # every run factors / updates the same inputs: as the reference re-generates them per run
        # (tests/testing_zpotrf.c:47-52), the operands are restored (untimed) before runs 2..nruns
        snap = [(M, M.data.clone()) for M in self.mats] if self.a.nruns > 1 else []
        for r in range(max(1, self.a.nruns)):
            if r > 0:
                for M, d in snap:
                    M.data.copy_(d)
                ctx.sync()
            ctx.barrier()
            t0 = time.perf_counter()
            tp = build()
            t_enq = time.perf_counter() - t0
            if getattr(self.a, "sim", False) and ctx.rank == 0:
                sim = getattr(tp, "simulation_date", None)
                print(f"{self.prec}{opname} simulation M= {self.a.M or self.a.N} N= {self.a.N} "
                      f"NB= {self.a.NB or self.a.MB} : {sim() if sim else 'n/a (not a tile-DAG taskpool)'}",
                      flush=True)
            ctx.barrier()
            ctx.sync()
            t1 = time.perf_counter()
            tp.run(ctx)
            res = tp.complete(ctx)
            ctx.sync()
            ctx.barrier()
            t2 = time.perf_counter()
            if ctx.profiling is not None:
                ctx.profiling.save_info(f"{opname}:TIME_ELAPSED", t2 - t1)
                ctx.profiling.save_info(f"{opname}:GFLOPS", tp.flops / max(t2 - t1, 1e-12) / 1e9)
            tp.destruct()
            t3 = time.perf_counter()
            self.report(opname, t2 - t1, tp.flops, t_enq, t3 - t2)
        return res

    def check(self, label, value, threshold):
        good = value < threshold and not math.isnan(value)
        self.ok &= good
        if self.ctx.rank == 0:
            print(f"-- {label} = {value:e} (threshold {threshold:g}): Solution is "
                  f"{'CORRECT' if good else 'SUSPICIOUS'}", flush=True)


# ----------------------------------------------------------------------------- operations
def t_potrf(h, dtd=False, untied=False):
    dp, a, ctx = h.dp, h.a, h.ctx
    uplo = dp.dplasmaLower if a.uplo.upper() == "L" else dp.dplasmaUpper
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, float(a.N), dp.dplasmaUpperLower, A, a.seed)
    A0 = A.like()
    A0.data.copy_(A.data)
    fn = dp.potrf_dtd_untied_New if untied else (dp.potrf_dtd_New if dtd else dp.potrf_New)
    name = "potrf_dtd_untied" if untied else ("potrf_dtd" if dtd else "potrf")
    info = h.run_tp(name, lambda: fn(ctx, uplo, A))
    if a.check:
        ok, res = dp.check_potrf(ctx, uplo, A, A0)
        h.check("||L L^H - A|| / (||A|| N eps)", res, 60.0)
    return info


def t_posv(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    K = a.K or 1
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, float(a.N), dp.dplasmaUpperLower, A, a.seed)
    A0 = A.like()
    A0.data.copy_(A.data)
    B = h.mat(a.N, K, name="B")
    dp.plrnt(ctx, B, a.seed + 1)
    B0 = B.like()
    B0.data.copy_(B.data)
    h.run_tp("posv", lambda: dp.posv_New(ctx, dp.dplasmaLower, A, B))
    if a.check:
        ok, res = dp.check_axmb(ctx, A0, B, B0)
        h.check("||Ax-b|| / ((||A|| ||x|| + ||b||) N eps)", res, 60.0)


def t_gemm(h, dtd=False):
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N, K = a.M or a.N, a.N, a.K or a.N
    A, B, C = h.mat(M, K, name="A"), h.mat(K, N, name="B"), h.mat(M, N, name="C")
    dp.plrnt(ctx, A, a.seed)
    dp.plrnt(ctx, B, a.seed + 1)
    dp.plrnt(ctx, C, a.seed + 2)
    if a.check:
        a_, b_, c_ = (_dense(h, X) for X in (A, B, C))
    fn = dp.gemm_dtd_New if dtd else dp.gemm_New
    h.run_tp("gemm_dtd" if dtd else "gemm", lambda: fn(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, a.alpha, A, B, 0.5, C))
    if a.check:
        ref = a.alpha * (a_ @ b_) + 0.5 * c_
        got = _dense(h, C)
        res = float((got - ref).abs().max() / (ref.abs().max() * K * EPS[h.prec]))
        h.check("||C - C_ref|| / (||C_ref|| K eps)", res, 10.0)


def t_trsm(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.K or a.N
    A, B = h.mat(M, M, name="A"), h.mat(M, N, name="B")
    dp.plghe(ctx, float(M), dp.dplasmaUpperLower, A, a.seed)
    dp.plrnt(ctx, B, a.seed + 1)
    b0 = _dense(h, B) if a.check else None
    a0 = _dense(h, A) if a.check else None
    h.run_tp("trsm", lambda: dp.trsm_New(ctx, dp.dplasmaLeft, dp.dplasmaLower, dp.dplasmaNoTrans,
                                          dp.dplasmaNonUnit, a.alpha, A, B))
    if a.check:
        x = _dense(h, B)
        res = float((torch.tril(a0) @ x - a.alpha * b0).abs().max() / (a0.abs().max() * x.abs().max() * M
                                                                         * EPS[h.prec] + 1e-300))
        h.check("||A X - alpha B|| / (||A|| ||X|| N eps)", res, 10.0)


def t_trmm(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.K or a.N
    A, B = h.mat(M, M, name="A"), h.mat(M, N, name="B")
    dp.plrnt(ctx, A, a.seed)
    dp.plrnt(ctx, B, a.seed + 1)
    a0, b0 = (_dense(h, A), _dense(h, B)) if a.check else (None, None)
    h.run_tp("trmm", lambda: dp.trmm_New(ctx, dp.dplasmaLeft, dp.dplasmaUpper, dp.dplasmaNoTrans,
                                          dp.dplasmaNonUnit, a.alpha, A, B))
    if a.check:
        ref = a.alpha * torch.triu(a0) @ b0
        res = float((_dense(h, B) - ref).abs().max() / (ref.abs().max() * M * EPS[h.prec]))
        h.check("||B - B_ref|| / (||B_ref|| N eps)", res, 10.0)


def _qr_common(h, lq, tree_kind, dtd=None):
    """testing_zgeqrf[_hqr|_systolic|_dtd|_dtd_untied|_rd].c and the LQ twins; dtd: "tied" / "untied" /
    "rd" (recursive-subtask hint, dplasma_zgeqrf_setrecursive)."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M = a.M or a.N
    N = a.N
    ib = a.IB or 32
    A = h.mat(M, N)
    if a.mtx:
        dp.pltmg(ctx, a.mtx, A, a.seed)
    else:
        dp.plrnt(ctx, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    TS = dp.block_cyclic(ctx, h.dt, ib, A.nb, A.mt * ib, A.nt * A.nb, name="TS")
    TT = dp.block_cyclic(ctx, h.dt, ib, A.nb, A.mt * ib, A.nt * A.nb, name="TT")
    trans = dp.dplasmaConjTrans if lq else dp.dplasmaNoTrans
    tree = None
    if tree_kind == "hqr":
        tree = dp.hqr_init(trans, A, a.treel, a.treeh, a.qr_a,
                           a.qr_p if a.qr_p > 0 else ctx.P, a.domino, a.tsrr)
    elif tree_kind == "systolic":
        tree = dp.systolic_init(trans, A, a.qr_p if a.qr_p > 0 else ctx.P, a.qr_a if a.qr_a > 0 else 1)
    if dtd in ("tied", "untied"):
        build = (lambda: dp.geqrf_dtd_New(ctx, A, TS)) if dtd == "tied" else \
            (lambda: dp.geqrf_dtd_untied_New(ctx, A, TS))
    elif dtd == "rd":
        def build():
            tp = dp.geqrf_New(ctx, A, TS)
            dp.geqrf_setrecursive(tp, a.HNB or max(1, A.nb // 2))
            return tp
    elif tree is None:
        build = (lambda: dp.gelqf_New(ctx, A, TS)) if lq else (lambda: dp.geqrf_New(ctx, A, TS))
    else:
        build = (lambda: dp.gelqf_param_New(ctx, tree, A, TS, TT)) if lq else \
            (lambda: dp.geqrf_param_New(ctx, tree, A, TS, TT))
    label = {"tied": "_dtd", "untied": "_dtd_untied", "rd": "_rd"}.get(dtd, "" if tree is None else "_" + tree_kind)
    h.run_tp(("gelqf" if lq else "geqrf") + label, build)
    if a.check:
        K = min(M, N)
        Q = h.mat(M if not lq else K, K if not lq else N, name="Q")
        if tree is None:
            (dp.unglq if lq else dp.ungqr)(ctx, A, TS, Q)
        else:
            (dp.unglq_param if lq else dp.ungqr_param)(ctx, tree, A, TS, TT, Q)
        q, r = _dense(h, Q), _dense(h, A)
        if not lq:
            orth = (q.conj().T @ q - torch.eye(K, dtype=q.dtype)).abs().max()
            rec = (q @ torch.triu(r[:K]) - a0).abs().max() / a0.abs().max()
        else:
            orth = (q @ q.conj().T - torch.eye(K, dtype=q.dtype)).abs().max()
            rec = (torch.tril(r[:, :K]) @ q - a0).abs().max() / a0.abs().max()
        h.check("||I - Q^H Q|| / (N eps)", float(orth) / (max(M, N) * EPS[h.prec]), 60.0)
        h.check("||A - Q R|| / (||A|| N eps)", float(rec) / (max(M, N) * EPS[h.prec]), 60.0)


def t_getrf(h, variant):
    dp, a, ctx = h.dp, h.a, h.ctx
    N = a.N
    A = h.mat(N, N)
    if variant == "nopiv":
        dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, a.seed)
    else:
        dp.plrnt(ctx, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    if variant in ("incpiv", "incpiv_dtd"):
        L = dp.incpiv_L_descriptor(ctx, A, a.IB or 32)
        IP = dp.incpiv_ipiv_descriptor(ctx, A)
        fn = dp.getrf_incpiv_dtd_New if variant == "incpiv_dtd" else dp.getrf_incpiv_New
        h.run_tp("getrf_" + variant, lambda: fn(ctx, A, L, IP))
    elif variant == "nopiv":
        h.run_tp("getrf_nopiv", lambda: dp.getrf_nopiv_New(ctx, A))
    else:
        IP = dp.ptgpanel_ipiv_descriptor(ctx, A)
        h.run_tp("getrf_" + variant, lambda: dp.getrf_ptgpanel_New(ctx, A, IP))
    if a.check:
        B = h.mat(N, a.K or 1, name="B")
        dp.plrnt(ctx, B, a.seed + 1)
        b0 = _dense(h, B)
        if variant in ("incpiv", "incpiv_dtd"):
            dp.trsmpl_incpiv(ctx, A, L, IP, B)
        elif variant == "nopiv":
            dp.trsm(ctx, dp.dplasmaLeft, dp.dplasmaLower, dp.dplasmaNoTrans, dp.dplasmaUnit, 1.0, A, B)
        else:
            dp.trsmpl_ptgpanel(ctx, A, IP, B)
        dp.trsm(ctx, dp.dplasmaLeft, dp.dplasmaUpper, dp.dplasmaNoTrans, dp.dplasmaNonUnit, 1.0, A, B)
        x = _dense(h, B)
        res = float(_inf(a0 @ x - b0) / ((_inf(a0) * _inf(x) + _inf(b0)) * N
                                                  * EPS[h.prec]))
        h.check("||Ax-b|| / ((||A|| ||x|| + ||b||) N eps)", res, 60.0)


def t_lange(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.N
    A = h.mat(M, N)
    dp.plrnt(ctx, A, a.seed)
    d = _dense(h, A)
    for nm, code, ref in (("max", dp.dplasmaMaxNorm, d.abs().max()), ("one", dp.dplasmaOneNorm, d.abs().sum(0).max()),
                          ("inf", dp.dplasmaInfNorm, d.abs().sum(1).max()),
                          ("frb", dp.dplasmaFrobeniusNorm, torch.linalg.norm(d))):
        t0 = time.perf_counter()
        v = dp.lange(ctx, code, A)
        if ctx.rank == 0:
            print(f"[****] TIME(s) {time.perf_counter() - t0:12.5f} : {h.prec}lange({nm}) = {v:.15e}")
        if a.check:
            h.check(f"|lange({nm}) - ref| / (ref eps N)", abs(v - float(ref)) / (float(ref) * EPS[h.prec] * N), 10.0)


def t_lanm2(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    A = h.mat(a.M or a.N, a.N)
    dp.plrnt(ctx, A, a.seed)
    info = []
    t0 = time.perf_counter()
    v = dp.lanm2(ctx, A, info)
    if ctx.rank == 0:
        print(f"[****] TIME(s) {time.perf_counter() - t0:12.5f} : {h.prec}lanm2 = {v:.15e} (iterations {info[0]})")
    if a.check:
        ref = float(torch.linalg.matrix_norm(_dense(h, A).to(torch.complex128 if h.dt.is_complex else torch.float64),
                                             2))
        h.check("|lanm2 - ||A||_2| / ||A||_2", abs(v - ref) / ref, 1e-5)


def t_print(h):
    dp, a, ctx = h.dp, h.a, h.ctx
    A = h.mat(a.M or a.N, a.N)
    dp.plrnt(ctx, A, a.seed)
    dp.print(ctx, dp.dplasmaUpperLower, A)


def t_heev(h):
    """testing_zheev.c: eigenvalues of a Hermitian matrix vs LAPACK on the original."""
    dp, a, ctx = h.dp, h.a, h.ctx
    uplo = dp.dplasmaLower if a.uplo.upper() == "L" else dp.dplasmaUpper
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, 0.0, dp.dplasmaUpperLower, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    W = torch.zeros(a.N, dtype=torch.float64)
    ib = a.IB or min(32, A.nb)
    h.run_tp("heev", lambda: dp.heev_New(ctx, dp.dplasmaNoVec, uplo, A, W, ib=ib))
    if a.check:
        ref = torch.linalg.eigvalsh(a0.to(torch.complex128 if h.dt.is_complex else torch.float64))
        res = float((W - ref).abs().max() / (ref.abs().max() * a.N * EPS[h.prec]))
        h.check("max|w - w_lapack| / (||A|| N eps)", res, 60.0)


def t_gebrd_ge2gb(h):
    """testing_zgebrd_ge2gb.c: reduction to band bidiagonal; check its singular values."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = max(a.M or a.N, a.N), a.N
    A = h.mat(M, N)
    dp.plrnt(ctx, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    ib = a.IB or min(32, A.nb)
    tp_box = []

    def build():
        tp = dp.gebrd_ge2gb_New(ctx, ib, A)
        tp_box.append(tp)
        return tp
    h.run_tp("gebrd_ge2gb", build)
    if a.check:
        s = torch.from_numpy(dp.band_singular_values(tp_box[-1].band, A.nb).copy())
        ref = torch.linalg.svdvals(a0.to(torch.complex128 if h.dt.is_complex else torch.float64))
        res = float((s - ref).abs().max() / (ref.max() * max(M, N) * EPS[h.prec]))
        h.check("max|sigma - sigma_lapack| / (||A|| N eps)", res, 60.0)


def t_hetrf(h):
    """testing_zhebut.c: RBT + LDL^H without pivoting, then solve."""
    dp, a, ctx = h.dp, h.a, h.ctx
    K = a.K or 1
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, float(a.N), dp.dplasmaUpperLower, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    B = h.mat(a.N, K, name="B")
    dp.plrnt(ctx, B, a.seed + 1)
    b0 = _dense(h, B) if a.check else None
    levels = 2 if a.N % 4 == 0 else 0
    U = dp.hebut(ctx, A, levels) if levels else None
    h.run_tp("hetrf", lambda: dp.hetrf_New(ctx, A))
    dp.hetrs(ctx, A, B, U)
    if a.check:
        x = _dense(h, B)
        res = float(_inf(a0 @ x - b0) / ((_inf(a0) * _inf(x) + _inf(b0)) * a.N
                                                  * EPS[h.prec]))
        h.check("||Ax-b|| / ((||A|| ||x|| + ||b||) N eps)", res, 60.0)


def t_getrf_qrf(h):
    """testing_zgetrf_qrf.c: hybrid LU-QR, then trsmpl_qrf + trsm(U) solve check."""
    dp, a, ctx = h.dp, h.a, h.ctx
    A = h.mat(a.N, a.N)
    dp.plrnt(ctx, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    ib = a.IB or min(32, A.nb)
    TS = h.mat(A.mt * ib, a.N, mb=ib, nb=A.nb, name="TS")
    TT = h.mat(A.mt * ib, a.N, mb=ib, nb=A.nb, name="TT")
    IP = dp.qrf_ipiv_descriptor(ctx, A)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, a.treel, a.treeh, a.qr_a,
                       a.qr_p if a.qr_p > 0 else ctx.P, a.domino, a.tsrr)
    lu_tab = [0] * min(A.mt, A.nt)
    h.run_tp("getrf_qrf", lambda: dp.getrf_qrf_New(ctx, tree, A, IP, TS, TT, a.criteria, a.alpha, lu_tab))
    if ctx.rank == 0:
        print(f"-- lu_tab: {' '.join(map(str, lu_tab))}  ({sum(lu_tab)} LU / {len(lu_tab)} steps)")
    if a.check:
        B = h.mat(a.N, a.K or 1, name="B")
        dp.plrnt(ctx, B, a.seed + 1)
        b0 = _dense(h, B)
        dp.trsmpl_qrf(ctx, tree, A, IP, B, TS, TT, lu_tab)
        dp.trsm(ctx, dp.dplasmaLeft, dp.dplasmaUpper, dp.dplasmaNoTrans, dp.dplasmaNonUnit, 1.0, A, B)
        x = _dense(h, B)
        res = float(_inf(a0 @ x - b0) / ((_inf(a0) * _inf(x) + _inf(b0)) * a.N
                                                  * EPS[h.prec]))
        h.check("||Ax-b|| / ((||A|| ||x|| + ||b||) N eps)", res, 60.0)


# ----------------------------------------------------------------------------- level-3 BLAS (reference comparison)
def _uplo(h):
    return h.dp.dplasmaLower if h.a.uplo.upper() == "L" else h.dp.dplasmaUpper


def _full_from(d, lower, herm):
    """The symmetric / Hermitian matrix whose `lower` (or upper) triangle is stored in d."""
    t = torch.tril(d) if lower else torch.triu(d)
    o = (torch.tril(d, -1) if lower else torch.triu(d, 1)).T
    full = t + (o.conj() if herm else o)
    if herm and full.is_complex():
        full.diagonal().imag.zero_()
    return full


def _blas_check(h, got, ref, K):
    res = float((got - ref).abs().max() / (ref.abs().max() * max(K, 1) * EPS[h.prec] + 1e-300))
    h.check("||C - C_ref|| / (||C_ref|| K eps)", res, 10.0)


def t_hemm(h, herm=True):
    """testing_zhemm.c / testing_zsymm.c: C = alpha A B + beta C, A Hermitian/symmetric (left side)."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.N
    uplo = _uplo(h)
    A, B, C = h.mat(M, M, name="A"), h.mat(M, N, name="B"), h.mat(M, N, name="C")
    dp.plrnt(ctx, A, a.seed)
    dp.plrnt(ctx, B, a.seed + 1)
    dp.plrnt(ctx, C, a.seed + 2)
    if a.check:
        a_, b_, c_ = (_dense(h, X) for X in (A, B, C))
    fn = dp.hemm_New if herm else dp.symm_New
    h.run_tp("hemm" if herm else "symm", lambda: fn(ctx, dp.dplasmaLeft, uplo, a.alpha, A, B, 0.5, C))
    if a.check:
        ref = a.alpha * (_full_from(a_, uplo == dp.dplasmaLower, herm) @ b_) + 0.5 * c_
        _blas_check(h, _dense(h, C), ref, M)


def t_herk(h, herm=True, two=False):
    """testing_z{herk,syrk,her2k,syr2k}.c: C = alpha A A^H (+ B A^H ...) + beta C on the `uplo` triangle."""
    dp, a, ctx = h.dp, h.a, h.ctx
    N, K = a.N, a.K or a.N
    uplo = _uplo(h)
    A, C = h.mat(N, K, name="A"), h.mat(N, N, name="C")
    B = h.mat(N, K, name="B") if two else None
    dp.plrnt(ctx, A, a.seed)
    if two:
        dp.plrnt(ctx, B, a.seed + 1)
    dp.plghe(ctx, 0.0, dp.dplasmaUpperLower, C, a.seed + 2)
    if a.check:
        a_, c_ = _dense(h, A), _dense(h, C)
        b_ = _dense(h, B) if two else None
    op = (lambda x: x.conj().T) if herm else (lambda x: x.T)
    name = ("her2k" if two else "herk") if herm else ("syr2k" if two else "syrk")
    fn = getattr(dp, name + "_New")
    if two:
        h.run_tp(name, lambda: fn(ctx, uplo, dp.dplasmaNoTrans, a.alpha, A, B, 0.5, C))
    else:
        h.run_tp(name, lambda: fn(ctx, uplo, dp.dplasmaNoTrans, a.alpha, A, 0.5, C))
    if a.check:
        prod = a_ @ op(b_) + b_ @ op(a_) if two else a_ @ op(a_)
        ref = a.alpha * prod + 0.5 * c_
        mask = torch.ones(N, N, dtype=torch.bool)
        mask = torch.tril(mask) if uplo == dp.dplasmaLower else torch.triu(mask)
        got = _dense(h, C)
        _blas_check(h, torch.where(mask, got, torch.zeros_like(got)), torch.where(mask, ref, torch.zeros_like(ref)),
                    K)


def t_geadd(h):
    """testing_zgeadd.c: B = alpha op(A) + beta B."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.N
    A, B = h.mat(M, N, name="A"), h.mat(M, N, name="B")
    dp.plrnt(ctx, A, a.seed)
    dp.plrnt(ctx, B, a.seed + 1)
    if a.check:
        a_, b_ = _dense(h, A), _dense(h, B)
    h.run_tp("geadd", lambda: dp.geadd_New(ctx, dp.dplasmaNoTrans, a.alpha, A, 0.5, B))
    if a.check:
        _blas_check(h, _dense(h, B), a.alpha * a_ + 0.5 * b_, 1)


# ----------------------------------------------------------------------------- inverses
def t_trtri(h):
    """testing_ztrtri.c: inverse of a triangular matrix, ||I - A^-1 A||."""
    dp, a, ctx = h.dp, h.a, h.ctx
    uplo = _uplo(h)
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, float(a.N), dp.dplasmaUpperLower, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    h.run_tp("trtri", lambda: dp.trtri_New(ctx, uplo, dp.dplasmaNonUnit, A))
    if a.check:
        tri = torch.tril if uplo == dp.dplasmaLower else torch.triu
        res = float((tri(_dense(h, A)) @ tri(a0) - torch.eye(a.N, dtype=a0.dtype)).abs().max()
                    / (a.N * EPS[h.prec]))
        h.check("||I - A^-1 A|| / (N eps)", res, 60.0 * float(tri(a0).abs().max()))


def t_poinv(h):
    """testing_zpoinv.c: inverse of an SPD matrix (potrf + trtri + lauum in one taskpool)."""
    dp, a, ctx = h.dp, h.a, h.ctx
    uplo = _uplo(h)
    A = h.mat(a.N, a.N)
    dp.plghe(ctx, float(a.N), dp.dplasmaUpperLower, A, a.seed)
    a0 = _dense(h, A) if a.check else None
    h.run_tp("poinv", lambda: dp.poinv_New(ctx, uplo, A))
    if a.check:
        inv = _full_from(_dense(h, A), uplo == dp.dplasmaLower, True)
        res = float((inv @ a0 - torch.eye(a.N, dtype=a0.dtype)).abs().max()
                    / (a0.abs().max() * inv.abs().max() * a.N * EPS[h.prec]))
        h.check("||I - A^-1 A|| / (||A|| ||A^-1|| N eps)", res, 60.0)


# ----------------------------------------------------------------------------- Q applications
def t_unmqr(h, lq, tree_kind):
    """testing_zunm{qr,lq}[_hqr|_systolic].c: C := op(Q) C and C op(Q) checked against the explicit Q."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M = a.M or a.N
    N = a.N
    K = a.K or N
    ib = a.IB or 32
    A = h.mat(M, N)
    dp.plrnt(ctx, A, a.seed)
    TS = dp.block_cyclic(ctx, h.dt, ib, A.nb, A.mt * ib, A.nt * A.nb, name="TS")
    TT = dp.block_cyclic(ctx, h.dt, ib, A.nb, A.mt * ib, A.nt * A.nb, name="TT")
    trans_t = dp.dplasmaConjTrans if lq else dp.dplasmaNoTrans
    tree = None
    if tree_kind == "hqr":
        tree = dp.hqr_init(trans_t, A, a.treel, a.treeh, a.qr_a,
                           a.qr_p if a.qr_p > 0 else ctx.P, a.domino, a.tsrr)
    elif tree_kind == "systolic":
        tree = dp.systolic_init(trans_t, A, a.qr_p if a.qr_p > 0 else ctx.P, a.qr_a if a.qr_a > 0 else 1)
    if tree is None:
        (dp.gelqf if lq else dp.geqrf)(ctx, A, TS)
    else:
        (dp.gelqf_param if lq else dp.geqrf_param)(ctx, tree, A, TS, TT)
    nq = N if lq else M          # Q is nq x nq
    Qm = h.mat(nq, nq, name="Q")
    if tree is None:
        (dp.unglq if lq else dp.ungqr)(ctx, A, TS, Qm)
    else:
        (dp.unglq_param if lq else dp.ungqr_param)(ctx, tree, A, TS, TT, Qm)
    q = _dense(h, Qm)
    name = ("unmlq" if lq else "unmqr") + ("" if tree is None else "_" + tree_kind)
    for side in (dp.dplasmaLeft, dp.dplasmaRight):
        for trans in (dp.dplasmaNoTrans, dp.dplasmaConjTrans):
            C = h.mat(nq, K, name="C") if side == dp.dplasmaLeft else h.mat(K, nq, name="C")
            dp.plrnt(ctx, C, a.seed + 3)
            c0 = _dense(h, C)
            if tree is None:
                build = lambda C=C, s=side, t=trans: (dp.unmlq_New if lq else dp.unmqr_New)(ctx, s, t, A, TS, C)  # noqa: E731
            else:
                build = lambda C=C, s=side, t=trans: (dp.unmlq_param_New if lq else dp.unmqr_param_New)(  # noqa: E731
                    ctx, s, t, tree, A, TS, TT, C)
            h.run_tp(name, build)
            if a.check:
                op = q if trans == dp.dplasmaNoTrans else q.conj().T
                ref = op @ c0 if side == dp.dplasmaLeft else c0 @ op
                res = float((_dense(h, C) - ref).abs().max() / (c0.abs().max() * nq * EPS[h.prec]))
                h.check(f"||{'L' if side == dp.dplasmaLeft else 'R'}{'N' if trans == dp.dplasmaNoTrans else 'C'}: "
                        f"op(Q) C - ref|| / (||C|| N eps)", res, 60.0)


# ----------------------------------------------------------------------------- solvers and reductions
def t_gesv_incpiv(h):
    """testing_zgesv_incpiv.c: A X = B with incremental-pivoting LU."""
    dp, a, ctx = h.dp, h.a, h.ctx
    N, K = a.N, a.K or 1
    A = h.mat(N, N)
    dp.plrnt(ctx, A, a.seed)
    B = h.mat(N, K, name="B")
    dp.plrnt(ctx, B, a.seed + 1)
    a0, b0 = (_dense(h, A), _dense(h, B)) if a.check else (None, None)
    L = dp.incpiv_L_descriptor(ctx, A, a.IB or 32)
    IP = dp.incpiv_ipiv_descriptor(ctx, A)
    t0 = time.perf_counter()
    info = dp.gesv_incpiv(ctx, A, L, IP, B)
    ctx.sync()
    from .utils.flops import flops
    h.report("gesv_incpiv", time.perf_counter() - t0, flops(A.prec, "getrf", N, N)
             + 2 * flops(A.prec, "trsm", True, N, K))
    if a.check:
        x = _dense(h, B)
        res = float(_inf(a0 @ x - b0) / ((_inf(a0) * _inf(x) + _inf(b0)) * N
                                                  * EPS[h.prec]))
        h.check("||Ax-b|| / ((||A|| ||x|| + ||b||) N eps)", res, 60.0)
    return info


def t_gesvd(h):
    """testing_zgesvd.c: singular values through the two-stage reduction (ge2gb to band, then the band
    bidiagonal's singular values) against LAPACK on the original matrix."""
    t_gebrd_ge2gb(h)


def t_hbrdt(h):
    """testing_zhbrdt.c: Hermitian band -> real tridiagonal (bulge chasing); eigenvalues preserved."""
    dp, a, ctx = h.dp, h.a, h.ctx
    N = a.N
    b = a.NB or a.MB or 8
    g = torch.Generator().manual_seed(a.seed)
    rdt = torch.float64
    dt = torch.complex128 if h.dt.is_complex else torch.float64
    dense = torch.randn(N, N, generator=g, dtype=rdt)
    if dt.is_complex:
        dense = torch.complex(dense, torch.randn(N, N, generator=g, dtype=rdt))
    dense = torch.tril(torch.triu(dense, -b), 0)
    herm = dense + torch.tril(dense, -1).conj().T
    herm.diagonal().imag.zero_() if dt.is_complex else None
    band = torch.zeros(b + 1, N, dtype=dt)
    for j in range(N):
        for i in range(j, min(N, j + b + 1)):
            band[i - j, j] = herm[i, j]
    t0 = time.perf_counter()
    d, e = dp.hbrdt(ctx, band.numpy(), b)
    h.report("hbrdt", time.perf_counter() - t0, 6.0 * N * N * b)
    if a.check:
        T = torch.diag(torch.as_tensor(d, dtype=rdt)) + torch.diag(torch.as_tensor(e, dtype=rdt).abs(), -1) \
            + torch.diag(torch.as_tensor(e, dtype=rdt).abs(), 1)
        w, ref = torch.linalg.eigvalsh(T), torch.linalg.eigvalsh(herm)
        res = float((w - ref).abs().max() / (ref.abs().max() * N * EPS["d"]))
        h.check("max|w(T) - w(A)| / (||A|| N eps)", res, 60.0)


def t_pivgen(h):
    """testing_zpivgen.c / TestsQRPivgen.cmake: validate the QR elimination trees (every tile killed once,
    by a live pivot, in a consistent order) over the low/high-level trees, domain sizes and domino."""
    dp, a, ctx = h.dp, h.a, h.ctx
    M, N = a.M or a.N, a.N
    A = h.mat(M, N)
    bad = 0
    count = 0
    t0 = time.perf_counter()
    for llvl in (0, 1, 2, 3, 4):
        for hlvl in (0, 1, 2, 3):
            for qa in (1, 2, 4):
                for dom in (False, True):
                    tree = dp.hqr_init(dp.dplasmaNoTrans, A, llvl, hlvl, qa, a.qr_p if a.qr_p > 0 else 2, dom,
                                       a.tsrr)
                    count += 1
                    bad += int(dp.qrtree_check(A, tree) != 0)
    for p in (1, 2, 3):
        count += 1
        bad += int(dp.qrtree_check(A, dp.systolic_init(dp.dplasmaNoTrans, A, p, 1)) != 0)
    h.report("pivgen", time.perf_counter() - t0, 0.0)
    if ctx.rank == 0:
        print(f"[****] pivgen: {count} trees checked on {A.mt} x {A.nt} tiles, {bad} invalid", flush=True)
    h.check("invalid trees", float(bad), 0.5)


def _inf(x) -> float:
    """Infinity norm (max row sum of |x|) -- the norm of the reference's solve checks
    (tests/testing_zgetrf_incpiv.c:176-203, src/dplasma_zcheck.c check_zaxmb)."""
    x = x if x.dim() == 2 else x.view(-1, 1)
    return float(x.abs().sum(1).max())


def _dense(h, X):
    d = X.to_dense_local().cpu()
    if h.ctx.world > 1:
        import torch.distributed as dist
        t = d.to(h.ctx.device)
        dist.all_reduce(t)
        d = t.cpu()
    return d


OPS = {
    "potrf": t_potrf, "potrf_dtd": lambda h: t_potrf(h, dtd=True), "posv": t_posv, "gemm": t_gemm,
    "potrf_dtd_untied": lambda h: t_potrf(h, untied=True), "gemm_dtd": lambda h: t_gemm(h, dtd=True),
    "trsm": t_trsm, "trmm": t_trmm,
    "geqrf": lambda h: _qr_common(h, False, None), "gelqf": lambda h: _qr_common(h, True, None),
    "geqrf_hqr": lambda h: _qr_common(h, False, "hqr"), "gelqf_hqr": lambda h: _qr_common(h, True, "hqr"),
    "geqrf_systolic": lambda h: _qr_common(h, False, "systolic"),
    "gelqf_systolic": lambda h: _qr_common(h, True, "systolic"),
    "getrf_1d": lambda h: t_getrf(h, "1d"), "getrf_ptgpanel": lambda h: t_getrf(h, "ptgpanel"),
    "getrf_incpiv": lambda h: t_getrf(h, "incpiv"), "getrf_nopiv": lambda h: t_getrf(h, "nopiv"),
    "lange": t_lange, "lanm2": t_lanm2, "print": t_print,
    "getrf_qrf": t_getrf_qrf, "heev": t_heev, "gebrd_ge2gb": t_gebrd_ge2gb, "hetrf": t_hetrf, "hebut": t_hetrf,
    # DTD / recursive QR and DTD incremental-pivoting LU
    "geqrf_dtd": lambda h: _qr_common(h, False, None, "tied"),
    "geqrf_dtd_untied": lambda h: _qr_common(h, False, None, "untied"),
    "geqrf_rd": lambda h: _qr_common(h, False, None, "rd"),
    "getrf_incpiv_dtd": lambda h: t_getrf(h, "incpiv_dtd"),
    # level-3 BLAS against a dense reference
    "hemm": t_hemm, "symm": lambda h: t_hemm(h, herm=False),
    "herk": t_herk, "syrk": lambda h: t_herk(h, herm=False),
    "her2k": lambda h: t_herk(h, two=True), "syr2k": lambda h: t_herk(h, herm=False, two=True),
    "geadd": t_geadd, "trtri": t_trtri, "poinv": t_poinv,
    # Q applications
    "unmqr": lambda h: t_unmqr(h, False, None), "unmlq": lambda h: t_unmqr(h, True, None),
    "unmqr_hqr": lambda h: t_unmqr(h, False, "hqr"), "unmlq_hqr": lambda h: t_unmqr(h, True, "hqr"),
    "unmqr_systolic": lambda h: t_unmqr(h, False, "systolic"),
    "unmlq_systolic": lambda h: t_unmqr(h, True, "systolic"),
    "gesv_incpiv": t_gesv_incpiv, "gesvd": t_gesvd, "hbrdt": t_hbrdt, "pivgen": t_pivgen,
}


def main(argv=None):
    a = _parse(argv if argv is not None else sys.argv[1:])
    h = Harness(a)
    fn = OPS.get(h.name)
    if fn is None:
        raise SystemExit(f"unknown operation {h.name}; available: {', '.join(sorted(OPS))}")
    fn(h)
    if a.trace:
        tr = h.dp.profiling_stop(h.ctx, a.trace)
        if h.ctx.rank == 0 and a.verbose:
            tr.print_summary()
    if h.ctx.world > 1:
        import torch.distributed as dist
        dist.barrier()
    return 0 if h.ok else 1


if __name__ == "__main__":
    sys.exit(main())
