/* C-ABI test of the extended entry points (tools/gen_capi.py EXT; reference src/include/dplasma/
 * dplasma_z.h:106-349 and qr_param.h:120-148): every call is made once from plain C with a residual or
 * structural check computed here.  usage: test_capi_ext <gpus>  (gpus = 0: CPU reference path) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dplasma.h"

static int fails = 0;
#define CHECK(c, what)                                                                \
  do {                                                                                \
    if (!(c)) {                                                                       \
      fprintf(stderr, "FAIL %s (line %d): %s\n", what, __LINE__, dplasma_last_error()); \
      ++fails;                                                                        \
    } else {                                                                          \
      printf("ok   %s\n", what);                                                      \
    }                                                                                 \
  } while (0)

static dplasma_context_t *ctx;
static const double EPS = 2.220446049250313e-16;

static dplasma_desc_t *mk(int mb, int nb, int m, int n) {
  return dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, mb, nb, m, n, 1, 1, dplasmaUpperLower);
}
static double *get(const dplasma_desc_t *A, int m, int n) {
  double *h = calloc((size_t)m * n, sizeof(double));
  dplasma_desc_get_lapack(A, h, m);
  return h;
}
static double amax(const double *a, size_t n) {
  double v = 0;
  for (size_t i = 0; i < n; ++i) v = fmax(v, fabs(a[i]));
  return v;
}
/* ||A x - b|| / ((||A|| ||x|| + ||b||) N eps), A n x n, x b n x nrhs (column-major) */
static double resid(const double *a, const double *x, const double *b, int n, int nrhs) {
  double r = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double s = -b[i + (size_t)c * n];
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)c * n];
      r = fmax(r, fabs(s));
    }
  return r / ((amax(a, (size_t)n * n) * amax(x, (size_t)n * nrhs) + amax(b, (size_t)n * nrhs)) * n * EPS);
}

int main(int argc, char **argv) {
  const int gpus = argc > 1 ? atoi(argv[1]) : 0;
  ctx = dplasma_init(1, gpus);
  if (!ctx) { fprintf(stderr, "init: %s\n", dplasma_last_error()); return 1; }
  const int N = 64, NB = 16, IB = 4, NRHS = 3, MT = N / NB;

  /* ---- QR trees: hqr / systolic / svd init, check, queries, printing */
  dplasma_desc_t *A = mk(NB, NB, N, N);
  dplasma_qrtree_t qt, st, vt;
  CHECK(dplasma_hqr_init(&qt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 2, 1, 0, 0) == 0, "hqr_init");
  CHECK(qt.mt == MT && qt.nt == MT && qt.a == 2, "hqr tree fields");
  CHECK(dplasma_qrtree_check(A, &qt) == 0, "qrtree_check (hqr)");
  int heads_ok = 1;
  for (int k = 0; k < MT; ++k) {
    const int nh = qt.getnbgeqrf(&qt, k);
    heads_ok = heads_ok && nh >= 1 && qt.getm(&qt, k, 0) >= k;
    for (int m = k + 1; m < MT; ++m) heads_ok = heads_ok && qt.currpiv(&qt, k, m) >= k && qt.currpiv(&qt, k, m) < m;
  }
  CHECK(heads_ok, "qrtree query callbacks");
  dplasma_qrtree_print_type(A, &qt);
  dplasma_qrtree_print_pivot(A, &qt);
  dplasma_qrtree_print_nbgeqrt(A, &qt);
  dplasma_qrtree_print_geqrt_k(A, &qt, 0);
  dplasma_qrtree_print_next_k(A, &qt, 0);
  dplasma_qrtree_print_prev_k(A, &qt, 0);
  int *perm = calloc((size_t)MT * MT, sizeof(int));
  dplasma_qrtree_print_perm(A, &qt, perm);
  CHECK(perm[0] == 0, "qrtree_print_perm");
  free(perm);
  CHECK(dplasma_systolic_init(&st, dplasmaNoTrans, A, 2, 1) == 0 && dplasma_qrtree_check(A, &st) == 0, "systolic_init");
  CHECK(dplasma_svd_init(&vt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, 1, 1, 1) == 0 && dplasma_qrtree_check(A, &vt) == 0,
        "svd_init");

  /* ---- HQR: geqrf_param + geqrs_param solve, ungqr_param orthogonality, unmqr_param */
  dplasma_dplrnt(ctx, 0, A, 3872ULL);
  double *a0 = get(A, N, N);
  dplasma_desc_t *B = mk(NB, NB, N, NRHS);
  dplasma_dplrnt(ctx, 0, B, 4674ULL);
  double *b0 = get(B, N, NRHS);
  dplasma_desc_t *TS = mk(IB, NB, MT * IB, N), *TT = mk(IB, NB, MT * IB, N);
  CHECK(dplasma_dgeqrf_param(ctx, &qt, A, TS, TT) == 0, "dgeqrf_param");
  CHECK(dplasma_dgeqrs_param(ctx, &qt, A, TS, TT, B) == 0, "dgeqrs_param");
  double *x = get(B, N, NRHS);
  double r = resid(a0, x, b0, N, NRHS);
  printf("geqrf_param + geqrs_param residual %.2f\n", r);
  CHECK(r < 60, "HQR least-squares solve residual");
  dplasma_desc_t *Q = mk(NB, NB, N, N);
  CHECK(dplasma_dungqr_param(ctx, &qt, A, TS, TT, Q) == 0, "dungqr_param");
  double *q = get(Q, N, N), orth = 0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += q[k + (size_t)i * N] * q[k + (size_t)j * N];
      orth = fmax(orth, fabs(s - (i == j)));
    }
  CHECK(orth < 1e-12, "ungqr_param: Q^T Q = I");
  /* Q^T applied to Q by unmqr_param gives I */
  CHECK(dplasma_dunmqr_param(ctx, dplasmaLeft, dplasmaTrans, &qt, A, TS, TT, Q) == 0, "dunmqr_param");
  double *qi = get(Q, N, N), ierr = 0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) ierr = fmax(ierr, fabs(qi[i + (size_t)j * N] - (i == j)));
  CHECK(ierr < 1e-12, "unmqr_param: Q^T Q = I");
  free(q); free(qi); free(x);
  /* the _New / _Destruct form of geqrf_param */
  dplasma_dplrnt(ctx, 0, A, 3872ULL);
  dplasma_taskpool_t *tp = dplasma_dgeqrf_param_New(ctx, &qt, A, TS, TT);
  CHECK(tp && dplasma_context_add_taskpool(ctx, tp) == 0 && dplasma_context_start(ctx) == 0 &&
            dplasma_context_wait(ctx) == 0, "dgeqrf_param_New");
  dplasma_dgeqrf_param_Destruct(tp);

  /* ---- LQ with a tree: gelqf_param + gelqs_param, unglq_param, unmlq_param */
  dplasma_qrtree_t lt;
  dplasma_dplrnt(ctx, 0, A, 51ULL);
  double *a1 = get(A, N, N);
  dplasma_dplrnt(ctx, 0, B, 52ULL);
  double *b1 = get(B, N, NRHS);
  CHECK(dplasma_hqr_init(&lt, dplasmaConjTrans, A, DPLASMA_FLAT_TREE, DPLASMA_FLAT_TREE, 1, 1, 0, 0) == 0, "hqr_init (LQ)");
  dplasma_desc_t *TSl = mk(IB, NB, MT * IB, N), *TTl = mk(IB, NB, MT * IB, N);
  CHECK(dplasma_dgelqf_param(ctx, &lt, A, TSl, TTl) == 0, "dgelqf_param");
  CHECK(dplasma_dgelqs_param(ctx, &lt, A, TSl, TTl, B) == 0, "dgelqs_param");
  x = get(B, N, NRHS);
  r = resid(a1, x, b1, N, NRHS);
  printf("gelqf_param + gelqs_param residual %.2f\n", r);
  CHECK(r < 60, "LQ tree solve residual");
  CHECK(dplasma_dunglq_param(ctx, &lt, A, TSl, TTl, Q) == 0, "dunglq_param");
  CHECK(dplasma_dunmlq_param(ctx, dplasmaRight, dplasmaTrans, &lt, A, TSl, TTl, Q) == 0, "dunmlq_param");
  qi = get(Q, N, N);
  ierr = 0;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) ierr = fmax(ierr, fabs(qi[i + (size_t)j * N] - (i == j)));
  CHECK(ierr < 1e-12, "unglq_param + unmlq_param: Q Q^T = I");
  free(qi); free(x);

  /* ---- hybrid LU-QR: getrf_qrf + trsmpl_qrf + upper solve */
  dplasma_dplrnt(ctx, 0, A, 7ULL);
  double *a2 = get(A, N, N);
  dplasma_dplrnt(ctx, 0, B, 8ULL);
  double *b2 = get(B, N, NRHS);
  dplasma_desc_t *IPQ = dplasma_desc_ipiv(ctx, NB, 1, MT * NB, MT, 1, 1);
  int lu_tab[4] = {-1, -1, -1, -1}, info = -7;
  const int rq = dplasma_dgetrf_qrf(ctx, &qt, A, IPQ, TS, TT, 0 /* default: alternate */, 1.0, lu_tab, &info);
  CHECK(rq == 0 && info == 0, "dgetrf_qrf");
  CHECK(lu_tab[0] == 0 && lu_tab[1] == 1 && lu_tab[2] == 0 && lu_tab[3] == 1, "getrf_qrf lu_tab written back");
  CHECK(dplasma_dtrsmpl_qrf(ctx, &qt, A, IPQ, B, TS, TT, lu_tab) == 0, "dtrsmpl_qrf");
  CHECK(dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B) == 0, "dtrsm (upper)");
  x = get(B, N, NRHS);
  r = resid(a2, x, b2, N, NRHS);
  printf("getrf_qrf + trsmpl_qrf residual %.2f\n", r);
  CHECK(r < 60, "LU-QR solve residual");
  free(x);

  /* ---- incremental pivoting and ptgpanel forward solves */
  dplasma_dplrnt(ctx, 0, A, 9ULL);
  dplasma_dplrnt(ctx, 0, B, 10ULL);
  dplasma_desc_t *L = mk(IB, NB, MT * IB, N), *IPI = dplasma_desc_ipiv(ctx, NB, 1, N, MT, 1, 1);
  double *a3 = get(A, N, N), *b3 = get(B, N, NRHS);
  CHECK(dplasma_dgetrf_incpiv(ctx, A, L, IPI) == 0, "dgetrf_incpiv");
  CHECK(dplasma_dtrsmpl_incpiv(ctx, A, L, IPI, B) == 0, "dtrsmpl_incpiv");
  dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B);
  x = get(B, N, NRHS);
  r = resid(a3, x, b3, N, NRHS);
  printf("getrf_incpiv + trsmpl_incpiv residual %.2f\n", r);
  CHECK(r < 60, "incpiv solve residual");
  free(x);
  dplasma_dplrnt(ctx, 0, A, 11ULL);
  dplasma_dplrnt(ctx, 0, B, 12ULL);
  double *a4 = get(A, N, N), *b4 = get(B, N, NRHS);
  dplasma_desc_t *IP1 = dplasma_desc_ipiv(ctx, 1, NB, 1, N, 1, 1);
  CHECK(dplasma_dgetrf_ptgpanel(ctx, A, IP1) == 0, "dgetrf_ptgpanel");
  CHECK(dplasma_dtrsmpl_ptgpanel(ctx, A, IP1, B) == 0, "dtrsmpl_ptgpanel");
  dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B);
  x = get(B, N, NRHS);
  r = resid(a4, x, b4, N, NRHS);
  printf("getrf_ptgpanel + trsmpl_ptgpanel residual %.2f\n", r);
  CHECK(r < 60, "ptgpanel solve residual");
  free(x);
  /* laswp: the pivots of the factorisation applied to the original right-hand side (P b) */
  dplasma_desc_set_lapack(B, b4, N);
  CHECK(dplasma_dlaswp(ctx, B, IP1, 1) == 0, "dlaswp");
  int *piv = calloc(N, sizeof(int));
  dplasma_desc_get_lapack(IP1, piv, 1);
  double *pb = get(B, N, NRHS), *ref = malloc(sizeof(double) * N * NRHS), lerr = 0;
  memcpy(ref, b4, sizeof(double) * N * NRHS);
  for (int i = 0; i < N; ++i) {
    const int p = piv[i] - 1;   /* 1-based global row */
    for (int c = 0; c < NRHS; ++c) {
      const double t = ref[i + c * N];
      ref[i + c * N] = ref[p + c * N];
      ref[p + c * N] = t;
    }
  }
  for (int i = 0; i < N * NRHS; ++i) lerr = fmax(lerr, fabs(pb[i] - ref[i]));
  CHECK(lerr == 0.0, "laswp = the pivots' row interchanges");
  free(piv); free(pb); free(ref);

  /* ---- LDL^H with random butterflies: hebut + hetrf + hetrs; trdsm / trmdm / gebut / gebmm */
  dplasma_desc_t *H = mk(NB, NB, N, N);
  dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, H, 5ULL);
  double *h0 = get(H, N, N);
  dplasma_dplrnt(ctx, 0, B, 13ULL);
  double *b5 = get(B, N, NRHS);
  double *U = NULL;
  CHECK(dplasma_dhebut(ctx, H, &U, 2) == 0 && U != NULL, "dhebut");
  CHECK(dplasma_dhetrf(ctx, H) == 0, "dhetrf");
  CHECK(dplasma_dhetrs(ctx, dplasmaLower, H, B, U, 2) == 0, "dhetrs");
  x = get(B, N, NRHS);
  r = resid(h0, x, b5, N, NRHS);
  printf("hebut + hetrf + hetrs residual %.2f\n", r);
  CHECK(r < 60, "LDL^H + butterflies solve residual");
  free(x);
  dplasma_desc_t *G = mk(NB, NB, N, N);
  dplasma_dplrnt(ctx, 0, G, 14ULL);
  CHECK(dplasma_dgebut(ctx, G, U, 2) == 0, "dgebut");
  CHECK(dplasma_dgebmm(ctx, B, U, 2, dplasmaTrans) == 0, "dgebmm");
  dplasma_but_free(U);
  dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, H, 6ULL);
  CHECK(dplasma_dhetrf(ctx, H) == 0 && dplasma_dtrmdm(ctx, H) == 0, "dtrmdm");
  CHECK(dplasma_dtrdsm(ctx, H, B) == 0, "dtrdsm");

  /* ---- eigen / band reductions: heev (trace of A = sum of eigenvalues), herbt, hbrdt, ge2gb(x) */
  dplasma_desc_t *S = mk(NB, NB, N, N), *W = mk(NB, NB, N, 1);
  dplasma_dplghe(ctx, 0.0, dplasmaUpperLower, S, 15ULL);
  double *s0 = get(S, N, N), tr = 0;
  for (int i = 0; i < N; ++i) tr += s0[i + (size_t)i * N];
  CHECK(dplasma_dheev(ctx, dplasmaNoVec, dplasmaLower, S, W, NULL) == 0, "dheev");
  double *w = get(W, N, 1), sw = 0;
  for (int i = 0; i < N; ++i) sw += w[i];
  CHECK(fabs(sw - tr) < 1e-9 * (1 + fabs(tr)), "heev: sum of eigenvalues = trace");
  dplasma_dplghe(ctx, 0.0, dplasmaUpperLower, S, 15ULL);
  dplasma_desc_t *T = mk(IB, NB, MT * IB, N);
  CHECK(dplasma_dherbt(ctx, dplasmaLower, IB, S, T) == 0, "dherbt");
  CHECK(dplasma_dhbrdt(ctx, S) == 0, "dhbrdt");
  dplasma_desc_t *R = mk(NB, NB, N, N), *Band = mk(NB, NB, 2 * NB, N);
  dplasma_dplrnt(ctx, 0, R, 16ULL);
  CHECK(dplasma_dgebrd_ge2gb(ctx, IB, R, Band) == 0, "dgebrd_ge2gb");
  dplasma_qrtree_t q2, l2;
  dplasma_dplrnt(ctx, 0, R, 17ULL);
  dplasma_hqr_init(&q2, dplasmaNoTrans, R, DPLASMA_FLAT_TREE, DPLASMA_FLAT_TREE, 1, 1, 0, 0);
  dplasma_desc_t *Rl = mk(NB, NB, N, N - NB);
  dplasma_hqr_init(&l2, dplasmaConjTrans, Rl, DPLASMA_FLAT_TREE, DPLASMA_FLAT_TREE, 1, 1, 0, 0);
  CHECK(dplasma_dgebrd_ge2gbx(ctx, IB, NULL, &q2, &l2, R, TS, TT, TSl, TTl, Band) == 0, "dgebrd_ge2gbx");
  dplasma_hqr_finalize(&q2);
  dplasma_hqr_finalize(&l2);

  /* ---- rank-1 updates: A += alpha x y^T */
  dplasma_desc_t *X = mk(NB, NB, N, 1), *Y = mk(NB, NB, N, 1);
  dplasma_dplrnt(ctx, 0, X, 18ULL);
  dplasma_dplrnt(ctx, 0, Y, 19ULL);
  dplasma_dplrnt(ctx, 0, G, 20ULL);
  double *g0 = get(G, N, N), *xv = get(X, N, 1), *yv = get(Y, N, 1);
  CHECK(dplasma_dgeru(ctx, 0.5, X, Y, G) == 0, "dgeru");
  double *g1 = get(G, N, N), gerr = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) gerr = fmax(gerr, fabs(g1[i + (size_t)j * N] - g0[i + (size_t)j * N] - 0.5 * xv[i] * yv[j]));
  CHECK(gerr < 1e-14, "geru: A + alpha x y^T");
  CHECK(dplasma_dgerc(ctx, -0.5, X, Y, G) == 0, "dgerc");
  double *g2 = get(G, N, N);
  gerr = 0;
  for (int i = 0; i < N * N; ++i) gerr = fmax(gerr, fabs(g2[i] - g0[i]));
  CHECK(gerr < 1e-14, "gerc undoes geru (real)");

  /* ---- generators, norms, printing */
  dplasma_desc_t *D = mk(NB, NB, N, N);
  CHECK(dplasma_dlaset(ctx, dplasmaUpperLower, 0.0, 3.0, D) == 0, "laset");
  int linfo = -1;
  const double n2 = dplasma_dlanm2(ctx, D, &linfo);
  printf("lanm2(3 I) = %.12f (info %d)\n", n2, linfo);
  CHECK(fabs(n2 - 3.0) < 1e-8 && linfo > 0, "lanm2 of 3 I (converged: info = iterations)");
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixMinij, D, 3872ULL) == 0, "dpltmg (minij)");
  double *dm = get(D, N, N);
  CHECK(dm[3 + 5 * N] == 4.0, "pltmg minij entry");
  CHECK(dplasma_dlatms(ctx, dplasmaGeneral, 10.0, D, 3872ULL) == 0, "dlatms");
  dplasma_desc_t *small = mk(4, 4, 4, 4);
  dplasma_dlaset(ctx, dplasmaUpperLower, 1.0, 2.0, small);
  CHECK(dplasma_dprint(ctx, dplasmaUpperLower, small) == 0, "dprint");

  /* ---- recursive sub-taskpool sizes on _New taskpools */
  dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, A, 21ULL);
  tp = dplasma_dpotrf_New(ctx, dplasmaLower, A);
  dplasma_dpotrf_setrecursive(tp, 8);
  CHECK(tp && dplasma_context_add_taskpool(ctx, tp) == 0 && dplasma_context_start(ctx) == 0 &&
            dplasma_context_wait(ctx) == 0 && dplasma_taskpool_result(tp) == 0, "dpotrf_setrecursive + _New");
  dplasma_dpotrf_Destruct(tp);
  dplasma_dplrnt(ctx, 0, A, 22ULL);
  dplasma_desc_t *Tq = mk(IB, NB, MT * IB, N);
  tp = dplasma_dgeqrf_New(ctx, A, Tq);
  dplasma_dgeqrf_setrecursive(tp, 8);
  CHECK(tp && dplasma_context_add_taskpool(ctx, tp) == 0 && dplasma_context_start(ctx) == 0 &&
            dplasma_context_wait(ctx) == 0, "dgeqrf_setrecursive + _New");
  dplasma_dgeqrf_Destruct(tp);

  dplasma_hqr_finalize(&qt);
  dplasma_hqr_finalize(&lt);
  dplasma_systolic_finalize(&st);
  dplasma_svd_finalize(&vt);
  dplasma_fini(ctx);
  printf("%s (%d failures)\n", fails ? "CAPI EXT FAIL" : "CAPI EXT OK", fails);
  return fails ? 2 : 0;
}
