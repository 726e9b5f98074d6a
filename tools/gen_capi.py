#!/usr/bin/env python3
"""Generate the C ABI of dplasma_amd (the reference's ``dplasma.h`` / ``dplasma_z.h`` surface).

Writes ``capi/include/dplasma.h`` (enums, opaque handles, one prototype per op and precision)
and ``capi/dplasma_ops.cpp`` (one forwarding wrapper per prototype).  The per-precision
templating that the reference does with tools/PrecisionGenerator (z -> c, d, s text
substitution) is done here from one op table.

Argument codes: E enum, D descriptor, S scalar of the op's precision (complex for c/z),
R real double, I int, U unsigned long long (seed).
"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

# (op, return 'i' | 'r', args, precisions, argument names)
OPS = [
    ("geadd", "i", "ESDSD", "sdcz", "trans alpha A beta B"),
    ("tradd", "i", "EESDSD", "sdcz", "uplo trans alpha A beta B"),
    ("gemm", "i", "EESDDSD", "sdcz", "transA transB alpha A B beta C"),
    ("hemm", "i", "EESDDSD", "cz", "side uplo alpha A B beta C"),
    ("symm", "i", "EESDDSD", "sdcz", "side uplo alpha A B beta C"),
    ("herk", "i", "EERDRD", "cz", "uplo trans alpha A beta C"),
    ("syrk", "i", "EESDSD", "sdcz", "uplo trans alpha A beta C"),
    ("her2k", "i", "EESDDRD", "cz", "uplo trans alpha A B beta C"),
    ("syr2k", "i", "EESDDSD", "sdcz", "uplo trans alpha A B beta C"),
    ("trmm", "i", "EEEESDD", "sdcz", "side uplo trans diag alpha A B"),
    ("trsm", "i", "EEEESDD", "sdcz", "side uplo trans diag alpha A B"),
    ("potrf", "i", "ED", "sdcz", "uplo A"),
    ("potrs", "i", "EDD", "sdcz", "uplo A B"),
    ("posv", "i", "EDD", "sdcz", "uplo A B"),
    ("potri", "i", "ED", "sdcz", "uplo A"),
    ("poinv", "i", "ED", "sdcz", "uplo A"),
    ("poinv_sync", "i", "ED", "sdcz", "uplo A"),
    ("potrf_rec", "i", "EDI", "sdcz", "uplo A hmb"),
    ("geqrf_rec", "i", "DDI", "sdcz", "A T hnb"),
    ("getrs_incpiv", "i", "EDDDD", "sdcz", "trans A L IPIV B"),
    ("trtri", "i", "EED", "sdcz", "uplo diag A"),
    ("lauum", "i", "ED", "sdcz", "uplo A"),
    ("getrf_nopiv", "i", "D", "sdcz", "A"),
    ("getrf_1d", "i", "DD", "sdcz", "A IPIV"),
    ("getrf_ptgpanel", "i", "DD", "sdcz", "A IPIV"),
    ("getrs", "i", "EDDD", "sdcz", "trans A IPIV B"),
    ("gesv_1d", "i", "DDD", "sdcz", "A IPIV B"),
    ("getrf_incpiv", "i", "DDD", "sdcz", "A L IPIV"),
    ("gesv_incpiv", "i", "DDDD", "sdcz", "A L IPIV B"),
    ("geqrf", "i", "DD", "sdcz", "A T"),
    ("gelqf", "i", "DD", "sdcz", "A T"),
    ("geqrs", "i", "DDD", "sdcz", "A T B"),
    ("gelqs", "i", "DDD", "sdcz", "A T B"),
    ("gels", "i", "EDDD", "sdcz", "trans A T B"),
    ("ungqr", "i", "DDD", "sdcz", "A T Q"),
    ("unglq", "i", "DDD", "sdcz", "A T Q"),
    ("unmqr", "i", "EEDDD", "sdcz", "side trans A T C"),
    ("unmlq", "i", "EEDDD", "sdcz", "side trans A T C"),
    ("lacpy", "i", "EDD", "sdcz", "uplo A B"),
    ("laset", "i", "ESSD", "sdcz", "uplo alpha beta A"),
    ("lascal", "i", "ESD", "sdcz", "uplo alpha A"),
    ("lange", "r", "ED", "sdcz", "ntype A"),
    ("lanhe", "r", "EED", "cz", "ntype uplo A"),
    ("lansy", "r", "EED", "sdcz", "ntype uplo A"),
    ("lantr", "r", "EEED", "sdcz", "ntype uplo diag A"),
    ("plrnt", "i", "IDU", "sdcz", "diagdom A seed"),
    ("plghe", "i", "REDU", "sdcz", "bump uplo A seed"),
    ("plgsy", "i", "SEDU", "sdcz", "bump uplo A seed"),
]
CTYPE = {"s": "float", "d": "double", "c": "dplasma_complex32_t", "z": "dplasma_complex64_t"}
PCODE = {"s": 2, "d": 3, "c": 4, "z": 5}
# operations of the interpreter-free engine (capi/native.cpp): arguments after (ctx, prec)
NATIVE = {
    "potrf": "uplo, A",
    "potrs": "uplo, A, B",
    "posv": "uplo, A, B",
    "gemm": "transA, transB, &alpha, A, B, &beta, C",
    "trsm": "side, uplo, trans, diag, &alpha, A, B",
    "plghe": "bump, uplo, A, seed",
    "plrnt": "diagdom, A, seed",
    "plgsy": "&bump, uplo, A, seed",
    "herk": "uplo, trans, alpha, A, beta, C",
    "syrk": "uplo, trans, &alpha, A, &beta, C",
    "geadd": "trans, &alpha, A, &beta, B",
    "tradd": "uplo, trans, &alpha, A, &beta, B",
    "lacpy": "uplo, A, B",
    "laset": "uplo, &alpha, &beta, A",
    "lascal": "uplo, &alpha, A",
    "lange": "ntype, A",
    "lantr": "ntype, uplo, diag, A",
    "trmm": "side, uplo, trans, diag, &alpha, A, B",
    "symm": "side, uplo, &alpha, A, B, &beta, C",
    "hemm": "side, uplo, &alpha, A, B, &beta, C",
    "lansy": "ntype, uplo, A",
    "lanhe": "ntype, uplo, A",
    "getrf_1d": "A, IPIV",
    "getrs": "trans, A, IPIV, B",
    "gesv_1d": "A, IPIV, B",
    "geqrf": "A, T",
    "unmqr": "side, trans, A, T, C",
    "ungqr": "A, T, Q",
    "geqrs": "A, T, B",
    "gels": "trans, A, T, B",
    "her2k": "uplo, trans, &alpha, A, B, beta, C",
    "syr2k": "uplo, trans, &alpha, A, B, &beta, C",
    "trtri": "uplo, diag, A",
    "lauum": "uplo, A",
    "potri": "uplo, A",
    "poinv": "uplo, A",
    "getrf_nopiv": "A",
    "gelqf": "A, T",
    "unmlq": "side, trans, A, T, C",
    "unglq": "A, T, Q",
    "gelqs": "A, T, B",
    "getrf_incpiv": "A, L, IPIV",
    "getrs_incpiv": "trans, A, L, IPIV, B",
    "gesv_incpiv": "A, L, IPIV, B",
}
# same operation natively under another name: the recursive-size hint only changes the reference's CPU
# task granularity; a 1 x 1 ptgpanel grid is the 1-D LU; the _sync variant is the blocking call
NATIVE_ALIAS = {
    "potrf_rec": ("potrf", "uplo, A"),
    "geqrf_rec": ("geqrf", "A, T"),
    "getrf_ptgpanel": ("getrf_1d", "A, IPIV"),
    "poinv_sync": ("poinv", "uplo, A"),
}


# Entry points of the reference API with arguments the main table cannot express (QR-tree handles,
# caller arrays, butterfly handles, taskpool setters): src/include/dplasma/dplasma_z.h:106-349 and
# qr_param.h:120-148.  Codes as OPS plus Q (dplasma_qrtree_t *), P (int * of the caller, written back),
# B (butterfly handle: {T} * in, {T} ** out) and K (dplasma_taskpool_t *).  Each forwards to the
# framework (dplasma_amd.capi.call "x:<p><op>" / new); native contexts refuse them (no native builder).
# (op, return, [(code, name)], precisions, has _New, C name override)
EXT = [
    ("geqrf_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT")], "sdcz", True),
    ("gelqf_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT")], "sdcz", True),
    ("unmqr_param", "i", [("E", "side"), ("E", "trans"), ("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"),
                          ("D", "C")], "sdcz", True),
    ("unmlq_param", "i", [("E", "side"), ("E", "trans"), ("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"),
                          ("D", "C")], "sdcz", True),
    ("ungqr_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"), ("D", "Q")], "sdcz", True),
    ("unglq_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"), ("D", "Q")], "sdcz", True),
    ("geqrs_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"), ("D", "B")], "sdcz", False),
    ("gelqs_param", "i", [("Q", "qrtree"), ("D", "A"), ("D", "TS"), ("D", "TT"), ("D", "B")], "sdcz", False),
    ("getrf_qrf", "i", [("Q", "qrtree"), ("D", "A"), ("D", "IPIV"), ("D", "TS"), ("D", "TT"), ("I", "criteria"),
                        ("R", "alpha"), ("P", "lu_tab"), ("P", "INFO")], "sdcz", True),
    ("trsmpl_qrf", "i", [("Q", "qrtree"), ("D", "A"), ("D", "IPIV"), ("D", "B"), ("D", "TS"), ("D", "TT"),
                         ("P", "lu_tab")], "sdcz", True),
    ("trsmpl_incpiv", "i", [("D", "A"), ("D", "L"), ("D", "IPIV"), ("D", "B")], "sdcz", True),
    ("trsmpl_ptgpanel", "i", [("D", "A"), ("D", "IPIV"), ("D", "B")], "sdcz", False),
    ("hebut", "i", [("D", "A"), ("B", "U_but_ptr"), ("I", "level")], "sdcz", False),
    ("hetrf", "i", [("D", "A")], "sdcz", True),
    ("hetrs", "i", [("E", "uplo"), ("D", "A"), ("D", "B"), ("B", "U_but_vec"), ("I", "level")], "sdcz", False),
    ("gebut", "i", [("D", "A"), ("B", "U_but_vec"), ("I", "level")], "sdcz", False),
    ("gebmm", "i", [("D", "A"), ("B", "U_but_vec"), ("I", "level"), ("E", "trans")], "sdcz", False),
    ("trdsm", "i", [("D", "A"), ("D", "B")], "sdcz", True),
    ("trmdm", "i", [("D", "A")], "sdcz", True),
    ("heev", "i", [("E", "jobz"), ("E", "uplo"), ("D", "A"), ("D", "W"), ("D", "Z")], "sdcz", True),
    ("herbt", "i", [("E", "uplo"), ("I", "ib"), ("D", "A"), ("D", "T")], "sdcz", True),
    ("hbrdt", "i", [("D", "A")], "sdcz", False),
    ("gebrd_ge2gb", "i", [("I", "ib"), ("D", "A"), ("D", "Band")], "sdcz", True),
    ("gebrd_ge2gbx", "i", [("I", "ib"), ("Q", "qrtre0"), ("Q", "qrtree"), ("Q", "lqtree"), ("D", "A"),
                           ("D", "TS0"), ("D", "TT0"), ("D", "TS"), ("D", "TT"), ("D", "Band")], "sdcz", True),
    ("geru", "i", [("S", "alpha"), ("D", "X"), ("D", "Y"), ("D", "A")], "sdcz", True),
    ("gerc", "i", [("S", "alpha"), ("D", "X"), ("D", "Y"), ("D", "A")], "sdcz", True),
    ("laswp", "i", [("D", "A"), ("D", "IPIV"), ("I", "inc")], "sdcz", False),
    ("lanm2", "r", [("D", "A"), ("P", "info")], "sdcz", False),
    ("pltmg", "i", [("E", "mtxtype"), ("D", "A"), ("U", "seed")], "sdcz", False),
    ("latms", "i", [("E", "mtxtype"), ("R", "cond"), ("D", "A"), ("U", "seed")], "sdcz", False),
    ("print", "i", [("E", "uplo"), ("D", "A")], "sdcz", False),
    ("potrf_setrecursive", "v", [("K", "tp"), ("I", "hmb")], "sdcz", False),
    ("geqrf_setrecursive", "v", [("K", "tp"), ("I", "hnb")], "sdcz", False),
]


# EXT entry points the interpreter-free engine also runs: op -> native call for precision code pc
NATIVE_EXT = {
    "geru": lambda pc: f"nat_ger(ctx, {pc}, 0, &alpha, X, Y, A)",
    "gerc": lambda pc: f"nat_ger(ctx, {pc}, 1, &alpha, X, Y, A)",
    "laswp": lambda pc: f"nat_laswp(ctx, {pc}, A, IPIV, inc)",
    "trsmpl_ptgpanel": lambda pc: f"nat_trsmpl_ptgpanel(ctx, {pc}, A, IPIV, B)",
    "trsmpl_incpiv": lambda pc: f"nat_trsmpl_incpiv(ctx, {pc}, A, L, IPIV, B)",
    "hetrf": lambda pc: f"nat_hetrf(ctx, {pc}, A)",
    "trdsm": lambda pc: f"nat_trdsm(ctx, {pc}, A, B)",
    "trmdm": lambda pc: f"nat_trmdm(ctx, {pc}, A)",
    # tree-driven QR / LQ (native_qrtree.cpp trees, native.cpp *_param builders)
    "geqrf_param": lambda pc: f"nat_geqrf_param(ctx, {pc}, qrtree, A, TS, TT)",
    "gelqf_param": lambda pc: f"nat_gelqf_param(ctx, {pc}, qrtree, A, TS, TT)",
    "unmqr_param": lambda pc: f"nat_unmqr_param(ctx, {pc}, side, trans, qrtree, A, TS, TT, C)",
    "unmlq_param": lambda pc: f"nat_unmlq_param(ctx, {pc}, side, trans, qrtree, A, TS, TT, C)",
    "ungqr_param": lambda pc: f"nat_ungqr_param(ctx, {pc}, qrtree, A, TS, TT, Q)",
    "unglq_param": lambda pc: f"nat_unglq_param(ctx, {pc}, qrtree, A, TS, TT, Q)",
    "geqrs_param": lambda pc: f"nat_geqrs_param(ctx, {pc}, qrtree, A, TS, TT, B)",
    "gelqs_param": lambda pc: f"nat_gelqs_param(ctx, {pc}, qrtree, A, TS, TT, B)",
    # hybrid LU-QR (native.cpp nat_getrf_qrf: predicated LU / QR branches after a host decision per step)
    "getrf_qrf": lambda pc: f"nat_getrf_qrf(ctx, {pc}, qrtree, A, IPIV, TS, TT, criteria, alpha, lu_tab, INFO)",
    "trsmpl_qrf": lambda pc: f"nat_trsmpl_qrf(ctx, {pc}, qrtree, A, IPIV, B, TS, TT, lu_tab)",
    # eigenvalues (native.cpp: two-sided panel reduction to band, host bulge chase + QL)
    "herbt": lambda pc: f"nat_herbt(ctx, {pc}, uplo, ib, A, T)",
    "hbrdt": lambda pc: f"nat_hbrdt(ctx, {pc}, A)",
    "heev": lambda pc: f"nat_heev(ctx, {pc}, jobz, uplo, A, W, Z)",
    "gebrd_ge2gb": lambda pc: f"nat_gebrd_ge2gb(ctx, {pc}, ib, A, Band)",
    "gebrd_ge2gbx": lambda pc: f"nat_gebrd_ge2gbx(ctx, {pc}, ib, qrtre0, qrtree, lqtree, A, TS0, TT0, TS, TT, Band)",
}
# EXT entry points the engine answers directly (a value, no program)
NATIVE_EXT_DIRECT = {
    "lanm2": lambda pc: f"nat_lanm2(ctx, {pc}, A, info)",
    "print": lambda pc: f"nat_print(ctx, {pc}, uplo, A)",
    "hetrs": lambda pc: f"nat_hetrs(ctx, {pc}, uplo, A, B, U_but_vec, level)",
    "gebmm": lambda pc: f"nat_gebmm(ctx, {pc}, A, U_but_vec, level, trans)",
    "gebut": lambda pc: f"nat_gebut(ctx, {pc}, A, U_but_vec, level)",
    "pltmg": lambda pc: f"nat_pltmg(ctx, {pc}, mtxtype, A, seed)",
    "latms": lambda pc: f"nat_latms(ctx, {pc}, mtxtype, cond, A, seed)",
}


def ext_ctype(code, p):
    T = CTYPE[p]
    return {"E": "dplasma_enum_t", "D": "dplasma_desc_t *", "S": T, "R": "double", "I": "int",
            "U": "unsigned long long", "Q": "dplasma_qrtree_t *", "P": "int *", "B": T + " *",
            "K": "dplasma_taskpool_t *"}[code]


def ext_conv(code, nm, p):
    if code == "D":
        return f"dpl_arg_desc({nm})"
    if code in "EI":
        return f"dpl_arg_int({nm})"
    if code == "U":
        return f"dpl_arg_u64({nm})"
    if code == "R":
        return f"dpl_arg_real({nm})"
    if code == "S":
        return f"dpl_arg_{'cplx' if p in 'cz' else 'real'}({nm})"
    if code == "Q":
        return f"dpl_arg_qrtree({nm})"
    if code == "P":
        return f"dpl_arg_ptr({nm})"
    if code == "B":   # the caller's host butterfly vector (level x n values of the precision), by address
        return f"dpl_arg_u64((unsigned long long)(uintptr_t){nm})"
    raise ValueError(code)


def gen_ext(h, cpp):
    """prototypes into h, wrappers into cpp (see EXT)"""
    h += ["", "/* ---- QR reduction trees (qr_param.h): caller-allocated, filled by an init function; the query",
          " * functions answer for the tree built by the framework (models/qrtree.py) */",
          "#define DPLASMA_QR_KILLED_BY_TS 0", "#define DPLASMA_QR_KILLED_BY_LOCALTREE 1",
          "#define DPLASMA_QR_KILLED_BY_DOMINO 2", "#define DPLASMA_QR_KILLED_BY_DISTTREE 3",
          "#define DPLASMA_FLAT_TREE 0", "#define DPLASMA_GREEDY_TREE 1", "#define DPLASMA_FIBONACCI_TREE 2",
          "#define DPLASMA_BINARY_TREE 3", "#define DPLASMA_GREEDY1P_TREE 4",
          "typedef struct dplasma_qrtree_s dplasma_qrtree_t;",
          "#ifndef DPLASMA_QRTREE_DEFINED",
          "#define DPLASMA_QRTREE_DEFINED",
          "struct dplasma_qrtree_s {",
          "    int (*getnbgeqrf)(const dplasma_qrtree_t *qrtree, int k);",
          "    int (*getm)(const dplasma_qrtree_t *qrtree, int k, int i);",
          "    int (*geti)(const dplasma_qrtree_t *qrtree, int k, int m);",
          "    int (*gettype)(const dplasma_qrtree_t *qrtree, int k, int m);",
          "    int (*currpiv)(const dplasma_qrtree_t *qrtree, int k, int m);",
          "    int (*nextpiv)(const dplasma_qrtree_t *qrtree, int k, int p, int m);",
          "    int (*prevpiv)(const dplasma_qrtree_t *qrtree, int k, int p, int m);",
          "    int mt, nt, a, p;",
          "    void *args;   /* the framework's tree */",
          "};",
          "#endif",
          "int  dplasma_hqr_init(dplasma_qrtree_t *qrtree, dplasma_enum_t trans, dplasma_desc_t *A, int type_llvl,",
          "                      int type_hlvl, int a, int p, int domino, int tsrr);",
          "void dplasma_hqr_finalize(dplasma_qrtree_t *qrtree);",
          "int  dplasma_systolic_init(dplasma_qrtree_t *qrtree, dplasma_enum_t trans, dplasma_desc_t *A, int p, int q);",
          "void dplasma_systolic_finalize(dplasma_qrtree_t *qrtree);",
          "int  dplasma_svd_init(dplasma_qrtree_t *qrtree, dplasma_enum_t trans, dplasma_desc_t *A, int type_hlvl,",
          "                      int p, int nbcores_per_node, int ratio);",
          "void dplasma_svd_finalize(dplasma_qrtree_t *qrtree);",
          "int  dplasma_qrtree_check(dplasma_desc_t *A, dplasma_qrtree_t *qrtree);",
          "void dplasma_qrtree_print_dag(dplasma_desc_t *A, dplasma_qrtree_t *qrtree, char *filename);",
          "void dplasma_qrtree_print_type(dplasma_desc_t *A, dplasma_qrtree_t *qrtree);",
          "void dplasma_qrtree_print_pivot(dplasma_desc_t *A, dplasma_qrtree_t *qrtree);",
          "void dplasma_qrtree_print_nbgeqrt(dplasma_desc_t *A, dplasma_qrtree_t *qrtree);",
          "void dplasma_qrtree_print_perm(dplasma_desc_t *A, dplasma_qrtree_t *qrtree, int *perm);",
          "void dplasma_qrtree_print_next_k(dplasma_desc_t *A, dplasma_qrtree_t *qrtree, int k);",
          "void dplasma_qrtree_print_prev_k(dplasma_desc_t *A, dplasma_qrtree_t *qrtree, int k);",
          "void dplasma_qrtree_print_geqrt_k(dplasma_desc_t *A, dplasma_qrtree_t *qrtree, int k);",
          "/* LDL^H butterflies: hebut returns, as the reference does, a malloc'd host vector of level x N values of",
          " * the precision (row l = the random diagonal of level l; complex: imaginary parts 0) that hetrs / gebut /",
          " * gebmm take, on native and framework contexts alike; release it with free() or dplasma_but_free */",
          "void dplasma_but_free(void *U_but_vec);",
          "/* ---- further entry points (dplasma_z.h:106-349); on a native context they return an error, except",
          " * geru / gerc / laswp / lanm2 (run natively) */"]
    for op, ret, args, precs, has_new, *_ in EXT:
        for p in precs:
            cargs = ", ".join(("dplasma_taskpool_t *tp" if c == "K" else
                               f"{ext_ctype(c, p)}{'*' if c == 'B' and op == 'hebut' else ''}"
                               f"{'' if ext_ctype(c, p).endswith('*') else ' '}{nm}") for c, nm in args)
            rt = {"i": "int", "r": "double", "v": "void"}[ret]
            if args[0][0] == "K":
                proto = f"{rt} dplasma_{p}{op}({cargs})"
            else:
                proto = f"{rt} dplasma_{p}{op}(dplasma_context_t *ctx, {cargs})"
            h.append(proto + ";")
            if has_new:
                nargs = cargs
                h.append(f"dplasma_taskpool_t *dplasma_{p}{op}_New(dplasma_context_t *ctx, {nargs});")
                h.append(f"void dplasma_{p}{op}_Destruct(dplasma_taskpool_t *tp);")
            # ---- wrappers
            conv = ", ".join(ext_conv(c, nm, p) for c, nm in args if c != "K")
            if op == "hebut":   # vector out: the framework returns its bytes, copied into a malloc'd array
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ if (dpl_native(ctx)) return nat_hebut(ctx, {PCODE[p]}, A, '
                           f'(void **)U_but_ptr, level); '
                           f'DplGil g; return dpl_call_bytes_out(ctx, "x:{p}{op}", (void **)U_but_ptr, '
                           f'{{dpl_arg_desc(A), dpl_arg_int(level)}}); }}')
                continue
            if args[0][0] == "K":
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ dpl_tp_setter(tp, "x:{p}{op}", {args[1][1]}); }}')
                continue
            if op in NATIVE_EXT_DIRECT:
                call = (f'dpl_call_real(ctx, "x:{p}{op}", {{{conv}}})' if ret == "r"
                        else f'dpl_call_int(ctx, "x:{p}{op}", {{{conv}}})')
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ if (dpl_native(ctx)) return {NATIVE_EXT_DIRECT[op](PCODE[p])}; '
                           f'DplGil g; return {call}; }}')
                continue
            if op in NATIVE_EXT:   # the interpreter-free engine runs it (capi/native.cpp)
                nat_call = NATIVE_EXT[op](PCODE[p])
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ if (dpl_native(ctx)) return nat_execute(ctx, {nat_call}); '
                           f'DplGil g; return dpl_call_int(ctx, "x:{p}{op}", {{{conv}}}); }}')
                if has_new:
                    cpp.append(f'extern "C" DPL_CAPI dplasma_taskpool_t *dplasma_{p}{op}_New(dplasma_context_t *ctx, '
                               f'{cargs}) {{ if (dpl_native(ctx)) return nat_wrap({nat_call}); '
                               f'DplGil g; return dpl_call_new(ctx, "x:{p}{op}", {{{conv}}}); }}')
                    cpp.append(f'extern "C" DPL_CAPI void dplasma_{p}{op}_Destruct(dplasma_taskpool_t *tp) '
                               '{ dplasma_taskpool_free(tp); }')
                continue
            if ret == "r":
                call = f'dpl_call_real(ctx, "x:{p}{op}", {{{conv}}})'
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ if (dpl_native(ctx)) return (nat_unsupported("{p}{op}"), NAN); '
                           f'DplGil g; return {call}; }}')
            else:
                call = f'dpl_call_int(ctx, "x:{p}{op}", {{{conv}}})'
                cpp.append(f'extern "C" DPL_CAPI {proto} {{ if (dpl_native(ctx)) return nat_unsupported("{p}{op}"); '
                           f'DplGil g; return {call}; }}')
            if has_new:
                cpp.append(f'extern "C" DPL_CAPI dplasma_taskpool_t *dplasma_{p}{op}_New(dplasma_context_t *ctx, {cargs}) '
                           f'{{ if (dpl_native(ctx)) {{ nat_unsupported("{p}{op}"); return nullptr; }} '
                           f'DplGil g; return dpl_call_new(ctx, "x:{p}{op}", {{{conv}}}); }}')
                cpp.append(f'extern "C" DPL_CAPI void dplasma_{p}{op}_Destruct(dplasma_taskpool_t *tp) '
                           '{ dplasma_taskpool_free(tp); }')


# blocking solves run as two programs: the solve only when the factorisation returned info == 0, so a
# failed factorisation leaves B untouched (reference: src/zposv_wrapper.c:102-104, zgesv_1d_wrapper.c)
TWO_PHASE = {
    "posv": ("potrf", "uplo, A", "potrs", "uplo, A, B"),
    "gesv_1d": ("getrf_1d", "A, IPIV", "getrs", "111 /* NoTrans */, A, IPIV, B"),
}


def enums():
    from dplasma_amd import constants as C
    out = []
    for k in dir(C):
        if k.startswith("dplasma") and isinstance(getattr(C, k), int):
            out.append((k, getattr(C, k)))
    return sorted(out, key=lambda kv: (kv[1], kv[0]))


def c_args(spec, names, p):
    res = []
    for code, nm in zip(spec, names):
        t = {"E": "dplasma_enum_t", "D": "dplasma_desc_t *", "S": CTYPE[p], "R": "double", "I": "int",
             "U": "unsigned long long"}[code]
        res.append(f"{t} {nm}" if not t.endswith("*") else f"{t}{nm}")
    return res


def main():
    inc = ROOT / "capi" / "include"
    inc.mkdir(parents=True, exist_ok=True)
    h = ["/* Generated by tools/gen_capi.py -- C ABI of dplasma_amd (MI355X).",
         " * Mirrors the reference API (src/include/dplasma/dplasma_z.h, constants.h): blocking",
         " * dplasma_<p><op>(ctx, ...) calls on opaque context / descriptor handles. */",
         "#ifndef DPLASMA_AMD_H", "#define DPLASMA_AMD_H", "#ifndef __cplusplus", "#include <complex.h>", "#endif",
         "#ifdef __cplusplus",
         'extern "C" {', "#endif", "",
         "typedef int dplasma_enum_t;",
         "#ifdef __cplusplus",
         "typedef __complex__ float dplasma_complex32_t;   /* GNU C++: ABI of C's float _Complex */",
         "typedef __complex__ double dplasma_complex64_t;",
         "#else",
         "typedef float _Complex dplasma_complex32_t;",
         "typedef double _Complex dplasma_complex64_t;",
         "#endif",
         "typedef struct dplasma_context_s dplasma_context_t;",
         "typedef struct dplasma_desc_s dplasma_desc_t;",
         "typedef struct dplasma_taskpool_s dplasma_taskpool_t;", ""]
    for k, v in enums():
        h.append(f"#define {k} {v}")
    h += ["", "#define DPLASMA_SUCCESS 0",
          "/* runtime (parsec_init / parsec_fini); gpus: 0 = CPU reference path, <0 = all visible */",
          "dplasma_context_t *dplasma_init(int nb_cores, int gpus);",
          "void dplasma_fini(dplasma_context_t *ctx);",
          "/* interpreter-free single-GPU context (capi/native.cpp): never starts Python; descriptors are",
          " * LAPACK-layout device buffers (dplasma_desc_block_cyclic allocates, _lapack wraps a device pointer,",
          " * P = Q = 1); the level-3 BLAS, Cholesky / LU / QR families, maps, norms and generators listed in",
          " * README run natively, every other operation returns an error (dplasma_last_error) */",
          "dplasma_context_t *dplasma_init_native(int device);",
          "/* interpreter-free multi-process context (capi/native_dist.cpp): rank of world processes, one GPU",
          " * each, on a P x (world / P) grid (rank = myrow * Q + mycol); descriptors are this rank's tiles of the",
          " * 2-D block-cyclic distribution in ScaLAPACK local layout, desc_set/get_lapack take the whole matrix;",
          " * the Cholesky family (potrf / potrs / posv / potri / poinv / trtri / lauum), LU with partial pivoting",
          " * (getrf_1d / getrs / gesv_1d), the level-3 BLAS (gemm, trsm, trmm, herk / syrk / her2k / syr2k,",
          " * symm / hemm), the generators, the element-wise maps and the norms run across the ranks; the",
          " * other operations return an error there.  Tiles move through RCCL (a GPU per rank) or node-local files (ranks sharing a",
          " * GPU); DPLASMA_NATIVE_TRANSPORT=rccl|file overrides.  rdv_dir: a fresh directory every rank can",
          " * reach (NULL: $DPLASMA_NATIVE_RDV) */",
          "dplasma_context_t *dplasma_init_native_dist(int device, int rank, int world, int P, const char *rdv_dir);",
          "int dplasma_python_active(void);   /* 1 once the embedded interpreter has been started */",
          "int dplasma_context_rank(const dplasma_context_t *ctx);",
          "int dplasma_context_world(const dplasma_context_t *ctx);",
          "/* 2-D block-cyclic descriptor (parsec_matrix_block_cyclic_init): prec = dplasmaRealFloat ..",
          " * dplasmaComplexDouble; P, Q <= 0 take the context grid; uplo = dplasmaUpperLower for general. */",
          "dplasma_desc_t *dplasma_desc_block_cyclic(dplasma_context_t *ctx, int prec, int mb, int nb, int m, int n,",
          "                                          int P, int Q, dplasma_enum_t uplo);",
          "dplasma_desc_t *dplasma_desc_ipiv(dplasma_context_t *ctx, int mb, int nb, int m, int n, int P, int Q);",
          "void dplasma_desc_destroy(dplasma_desc_t *A);",
          "/* host LAPACK-layout (column-major, lda) <-> local tiles */",
          "int dplasma_desc_set_lapack(dplasma_desc_t *A, const void *host, int lda);",
          "int dplasma_desc_get_lapack(const dplasma_desc_t *A, void *host, int lda);",
          "/* descriptor over caller-owned memory in ScaLAPACK local layout (column-major, lld; tiles of",
          " * the 2-D block-cyclic distribution with first process row/col ip/jq): device memory of the",
          " * context's GPU when on_device != 0 (zero copy), host memory on a CPU context */",
          "dplasma_desc_t *dplasma_desc_block_cyclic_lapack(dplasma_context_t *ctx, int prec, int mb, int nb, int m,",
          "                                                 int n, int P, int Q, int ip, int jq, void *data, int lld,",
          "                                                 int on_device);",
          "/* taskpools (parsec_taskpool_t): dplasma_<p><op>_New builds, add/start/wait run, _Destruct frees */",
          "int dplasma_context_add_taskpool(dplasma_context_t *ctx, dplasma_taskpool_t *tp);",
          "int dplasma_context_start(dplasma_context_t *ctx);",
          "int dplasma_context_wait(dplasma_context_t *ctx);",
          "int dplasma_taskpool_result(const dplasma_taskpool_t *tp);   /* info of a completed taskpool */",
          "void dplasma_taskpool_free(dplasma_taskpool_t *tp);",
          "/* ScaLAPACK layer (src/scalapack_wrappers): BLACS handle onto a context, F77 entry points */",
          "int dplasma_blacs_gridinit(dplasma_context_t *ctx);",
          "void parsec_init_wrapper_(void);",
          "void parsec_fini_wrapper_(void);",
          "int numroc_(int *n, int *nb, int *iproc, int *isrcproc, int *nprocs);",
          "void descinit_(int *desc, int *m, int *n, int *mb, int *nb, int *irsrc, int *icsrc, int *ictxt, int *lld,",
          "               int *info);",
          "void blacs_pinfo_(int *mypnum, int *nprocs);",
          "void blacs_get_(int *icontxt, int *what, int *val);",
          "void blacs_gridinit_(int *icontxt, const char *order, int *nprow, int *npcol);",
          "void blacs_gridinfo_(int *icontxt, int *nprow, int *npcol, int *myrow, int *mycol);",
          "void blacs_gridexit_(int *icontxt);"]
    for p in "sdcz":
        T = CTYPE[p]
        h += [f"void p{p}gemm_(const char *transa, const char *transb, int *m, int *n, int *k, {T} *alpha, {T} *a,",
              f"             int *ia, int *ja, int *desca, {T} *b, int *ib, int *jb, int *descb, {T} *beta, {T} *c,",
              "             int *ic, int *jc, int *descc);",
              f"void p{p}potrf_(const char *uplo, int *n, {T} *a, int *ia, int *ja, int *desca, int *info);",
              f"void p{p}getrf_(int *m, int *n, {T} *a, int *ia, int *ja, int *desca, int *ipiv, int *info);",
              f"void p{p}trsm_(const char *side, const char *uplo, const char *transa, const char *diag, int *m, int *n,",
              f"             {T} *alpha, {T} *a, int *ia, int *ja, int *desca, {T} *b, int *ib, int *jb, int *descb);",
              f"void p{p}trmm_(const char *side, const char *uplo, const char *transa, const char *diag, int *m, int *n,",
              f"             {T} *alpha, {T} *a, int *ia, int *ja, int *desca, {T} *b, int *ib, int *jb, int *descb);",
              f"void p{p}latsqr_(int *m, int *n, {T} *a, int *ia, int *ja, int *desca, {T} *tau, {T} *work, int *lwork,",
              "               int *info);"]
    h += ["/* last Python-side error message of this thread (\"\" if none) */",
          "const char *dplasma_last_error(void);", "",
          "/* dplasma_info_t string options (src/utils/dplasma_info.h) */",
          "#define DPLASMA_MAX_INFO_KEY 255", "#define DPLASMA_MAX_INFO_VAL 1024",
          "typedef struct dplasma_info_s *dplasma_info_t;",
          "int dplasma_info_create(dplasma_info_t *info);",
          "int dplasma_info_free(dplasma_info_t *info);",
          "int dplasma_info_set(dplasma_info_t info, const char *key, const char *value);",
          "int dplasma_info_delete(dplasma_info_t info, const char *key);",
          "int dplasma_info_get(dplasma_info_t info, const char *key, int valuelen, char *value, int *flag);",
          "int dplasma_info_get_nkeys(dplasma_info_t info, int *nkeys);",
          "int dplasma_info_get_nthkey(dplasma_info_t info, int n, char *key);", ""]
    cpp_head = ['extern "C" void dplasma_taskpool_free(dplasma_taskpool_t *tp);']
    cpp = ['// Generated by tools/gen_capi.py: one forwarding wrapper per C prototype of dplasma.h (native',
           '// contexts dispatch to capi/native.cpp or fail; the others forward to dplasma_amd).',
           '#include "capi_bridge.h"', "#include <cmath>", ""]
    from dplasma_amd import api as _api
    n_new = 0
    for op, ret, spec, precs, names in OPS:
        names = names.split()
        for p in precs:
            rt = "int" if ret == "i" else "double"
            args = ", ".join(["dplasma_context_t *ctx"] + c_args(spec, names, p))
            h.append(f"{rt} dplasma_{p}{op}({args});")
            conv = []
            for code, nm in zip(spec, names):
                if code == "D":
                    conv.append(f"dpl_arg_desc({nm})")
                elif code in "EI":
                    conv.append(f"dpl_arg_int({nm})")
                elif code == "U":
                    conv.append(f"dpl_arg_u64({nm})")
                elif code == "R":
                    conv.append(f"dpl_arg_real({nm})")
                else:
                    conv.append(f"dpl_arg_{'cplx' if p in 'cz' else 'real'}({nm})")
            call = f'dpl_call_{"int" if ret == "i" else "real"}(ctx, "{p}{op}", {{{", ".join(conv)}}})'
            nat = NATIVE.get(op)
            nop = op
            if nat is None and op in NATIVE_ALIAS:
                nop, nat = NATIVE_ALIAS[op]
            if nat is not None and ret == "r":   # norms: computed and returned directly
                pre = f"if (dpl_native(ctx)) return nat_{nop}(ctx, {PCODE[p]}, {nat}); "
                pre_new = ""
            elif nat is not None:
                nat_call = f"nat_{nop}(ctx, {PCODE[p]}, {nat})"
                pre = f"if (dpl_native(ctx)) return nat_execute(ctx, {nat_call}); "
                pre_new = f"if (dpl_native(ctx)) return nat_wrap({nat_call}); "
                if op in TWO_PHASE:
                    f1, a1, f2, a2 = TWO_PHASE[op]
                    pre = (f"if (dpl_native(ctx)) {{ const int info = nat_execute(ctx, nat_{f1}(ctx, {PCODE[p]}, {a1})); "
                           f"return info != 0 ? info : nat_execute(ctx, nat_{f2}(ctx, {PCODE[p]}, {a2})); }} ")
            else:
                miss = f'nat_unsupported("{p}{op}")'
                pre = (f"if (dpl_native(ctx)) return {miss}; " if ret == "i"
                       else f"if (dpl_native(ctx)) return ({miss}, NAN); ")
                pre_new = f"if (dpl_native(ctx)) {{ {miss}; return nullptr; }} "
            cpp.append(f"extern \"C\" DPL_CAPI {rt} dplasma_{p}{op}({args}) {{ {pre}DplGil g; return {call}; }}")
            if hasattr(_api, f"{p}{op}_New"):
                n_new += 1
                h.append(f"dplasma_taskpool_t *dplasma_{p}{op}_New({args});")
                h.append(f"void dplasma_{p}{op}_Destruct(dplasma_taskpool_t *tp);")
                cpp.append(f"extern \"C\" DPL_CAPI dplasma_taskpool_t *dplasma_{p}{op}_New({args}) "
                           f"{{ {pre_new}DplGil g; return dpl_call_new(ctx, \"{p}{op}\", {{{', '.join(conv)}}}); }}")
                cpp.append(f"extern \"C\" DPL_CAPI void dplasma_{p}{op}_Destruct(dplasma_taskpool_t *tp) "
                           "{ dplasma_taskpool_free(tp); }")
    ext_cpp = ['// Generated by tools/gen_capi.py: the EXT entry points (QR-tree handles, caller arrays, butterfly',
               '// vectors, taskpool setters) forwarded to dplasma_amd.capi ("x:<p><op>").',
               '#include "capi_bridge.h"', "#include <cmath>", "#include <cstdint>", "",
               'extern "C" void dplasma_taskpool_free(dplasma_taskpool_t *tp);']
    gen_ext(h, ext_cpp)
    (ROOT / "capi" / "dplasma_ext.cpp").write_text("\n".join(ext_cpp) + "\n")
    h += ["", "#ifdef __cplusplus", "}", "#endif", "#endif", ""]
    (inc / "dplasma.h").write_text("\n".join(h))
    cpp = cpp[:4] + cpp_head + cpp[4:]
    (ROOT / "capi" / "dplasma_ops.cpp").write_text("\n".join(cpp) + "\n")
    print(f"wrote {inc / 'dplasma.h'} and capi/dplasma_ops.cpp ({sum(len(o[3]) for o in OPS)} blocking entry points, "
          f"{n_new} _New/_Destruct pairs)")


if __name__ == "__main__":
    main()
