/* Multi-process interpreter-free C ABI (dplasma_init_native_dist, capi/native_dist.cpp): every rank of a
 * P x Q grid runs the distributed operation and a one-process native context runs the same operation on
 * the whole matrix; each rank compares ITS tiles of the result (the reference's testing_*.c checks run
 * per rank on the local tiles too).  Cholesky lower / upper (d, z), SUMMA GEMM (transpose variants, d, z),
 * a failing factorisation's info on every rank, the norms, the maps, the taskpool lifecycle, and an
 * operation without a distributed builder (a clean error).
 * usage: test_native_dist rank world P rdv_dir */
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dplasma.h"

static int fails = 0, rank = 0, world = 1, P = 1, Q = 1;
#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      printf("FAIL rank %d %s:%d ", rank, __FILE__, __LINE__); \
      printf(__VA_ARGS__);                                 \
      printf("\n");                                        \
      fails++;                                             \
    }                                                      \
  } while (0)

static dplasma_context_t *cd, *c1;

static dplasma_desc_t *mat(dplasma_context_t *ctx, int prec, int nb, int m, int n) {
  dplasma_desc_t *A = dplasma_desc_block_cyclic(ctx, prec, nb, nb, m, n, 0, 0, dplasmaUpperLower);
  if (!A) printf("rank %d desc: %s\n", rank, dplasma_last_error());
  return A;
}

/* max |X - Y| over this rank's tiles (uplo part: 'L', 'U' or 'A'), relative to max |Y| */
static double cmp_local(const void *X, const void *Y, int cplx, int m, int n, int nb, char part) {
  double err = 0, nrm = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      if ((i / nb) % P != rank / Q || (j / nb) % Q != rank % Q) continue;
      if ((part == 'L' && i < j) || (part == 'U' && i > j)) continue;
      const size_t o = i + (size_t)j * m;
      double d, y;
      if (cplx) {
        d = cabs(((const double complex *)X)[o] - ((const double complex *)Y)[o]);
        y = cabs(((const double complex *)Y)[o]);
      } else {
        d = fabs(((const double *)X)[o] - ((const double *)Y)[o]);
        y = fabs(((const double *)Y)[o]);
      }
      if (!(d <= err)) err = d;   /* NaN-propagating */
      if (y > nrm) nrm = y;
    }
  return nrm > 0 ? err / nrm : err;
}

static void test_potrf(int prec, char uplo, int n, int nb) {
  const int cplx = prec == dplasmaComplexDouble, es = cplx ? 16 : 8;
  const dplasma_enum_t u = uplo == 'L' ? dplasmaLower : dplasmaUpper;
  dplasma_desc_t *A = mat(cd, prec, nb, n, n), *B = mat(c1, prec, nb, n, n);
  void *X = calloc((size_t)n * n, es), *Y = calloc((size_t)n * n, es);
  CHECK(A && B, "descriptors");
  if (!A || !B) return;
  int r1, r2, i1, i2;
  if (cplx) {
    r1 = dplasma_zplghe(cd, (double)n, u, A, 3872);
    r2 = dplasma_zplghe(c1, (double)n, u, B, 3872);
    i1 = dplasma_zpotrf(cd, u, A);
    i2 = dplasma_zpotrf(c1, u, B);
  } else {
    r1 = dplasma_dplghe(cd, (double)n, u, A, 3872);
    r2 = dplasma_dplghe(c1, (double)n, u, B, 3872);
    i1 = dplasma_dpotrf(cd, u, A);
    i2 = dplasma_dpotrf(c1, u, B);
  }
  CHECK(r1 == 0 && r2 == 0, "plghe: %s", dplasma_last_error());
  CHECK(i1 == 0 && i2 == 0, "%cpotrf %c info %d / %d: %s", cplx ? 'z' : 'd', uplo, i1, i2, dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, X, n) == 0 && dplasma_desc_get_lapack(B, Y, n) == 0, "get_lapack");
  const double e = cmp_local(X, Y, cplx, n, n, nb, uplo);
  CHECK(e < 1e-11, "%cpotrf %c n=%d nb=%d: local tiles differ from one process by %.3e", cplx ? 'z' : 'd', uplo, n,
        nb, e);
  if (rank == 0) printf("%cpotrf %c n=%d nb=%d grid %dx%d: max rel diff %.2e\n", cplx ? 'z' : 'd', uplo, n, nb, P, Q, e);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
  free(X), free(Y);
}

static void test_gemm(int prec, int ta, int tb, int m, int n, int k, int nb) {
  const int cplx = prec == dplasmaComplexDouble, es = cplx ? 16 : 8;
  const int am = ta == dplasmaNoTrans ? m : k, an = ta == dplasmaNoTrans ? k : m;
  const int bm = tb == dplasmaNoTrans ? k : n, bn = tb == dplasmaNoTrans ? n : k;
  dplasma_desc_t *A[2], *B[2], *C[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, am, an), B[s] = mat(cx[s], prec, nb, bm, bn), C[s] = mat(cx[s], prec, nb, m, n);
    ok = ok && A[s] && B[s] && C[s];
  }
  CHECK(ok, "descriptors");
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc;
    if (cplx) {
      rc = dplasma_zplrnt(cx[s], 0, A[s], 11) | dplasma_zplrnt(cx[s], 0, B[s], 12) | dplasma_zplrnt(cx[s], 0, C[s], 13);
      rc |= dplasma_zgemm(cx[s], ta, tb, 1.5 - 0.25 * I, A[s], B[s], -0.5 + 0.75 * I, C[s]);
    } else {
      rc = dplasma_dplrnt(cx[s], 0, A[s], 11) | dplasma_dplrnt(cx[s], 0, B[s], 12) | dplasma_dplrnt(cx[s], 0, C[s], 13);
      rc |= dplasma_dgemm(cx[s], ta, tb, 1.5, A[s], B[s], -0.5, C[s]);
    }
    CHECK(rc == 0, "gemm (%s context): %s", s ? "one-process" : "distributed", dplasma_last_error());
  }
  void *X = calloc((size_t)m * n, es), *Y = calloc((size_t)m * n, es);
  CHECK(dplasma_desc_get_lapack(C[0], X, m) == 0 && dplasma_desc_get_lapack(C[1], Y, m) == 0, "get_lapack");
  const double e = cmp_local(X, Y, cplx, m, n, nb, 'A');
  CHECK(e < 1e-12, "%cgemm %d%d %dx%dx%d: local tiles differ by %.3e", cplx ? 'z' : 'd', ta, tb, m, n, k, e);
  if (rank == 0) printf("%cgemm %d/%d %dx%dx%d grid %dx%d: max rel diff %.2e\n", cplx ? 'z' : 'd', ta, tb, m, n, k, P, Q, e);
  for (int s = 0; s < 2; ++s) dplasma_desc_destroy(A[s]), dplasma_desc_destroy(B[s]), dplasma_desc_destroy(C[s]);
  free(X), free(Y);
}

/* distributed TRSM / TRMM: every rank's tiles of B equal the one-process engine's (A: the triangle of a
 * diagonally dominant Hermitian matrix, so every solve is well conditioned) */
static void test_trxm(int prec, int solve, int side, int uplo, int trans, int diag, int n, int nrhs, int nb) {
  const int cplx = prec == dplasmaComplexDouble, es = cplx ? 16 : 8;
  const int bm = side == dplasmaLeft ? n : nrhs, bn = side == dplasmaLeft ? nrhs : n;
  dplasma_desc_t *A[2], *B[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, n, n), B[s] = mat(cx[s], prec, nb, bm, bn);
    ok = ok && A[s] && B[s];
  }
  CHECK(ok, "descriptors");
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc;
    if (cplx) {
      rc = dplasma_zplghe(cx[s], (double)n, dplasmaUpperLower, A[s], 21) | dplasma_zplrnt(cx[s], 0, B[s], 22);
      rc |= solve ? dplasma_ztrsm(cx[s], side, uplo, trans, diag, 0.75 + 0.5 * I, A[s], B[s])
                  : dplasma_ztrmm(cx[s], side, uplo, trans, diag, 0.75 + 0.5 * I, A[s], B[s]);
    } else {
      rc = dplasma_dplghe(cx[s], (double)n, dplasmaUpperLower, A[s], 21) | dplasma_dplrnt(cx[s], 0, B[s], 22);
      rc |= solve ? dplasma_dtrsm(cx[s], side, uplo, trans, diag, 0.75, A[s], B[s])
                  : dplasma_dtrmm(cx[s], side, uplo, trans, diag, 0.75, A[s], B[s]);
    }
    CHECK(rc == 0, "%s (%s context): %s", solve ? "trsm" : "trmm", s ? "one-process" : "distributed",
          dplasma_last_error());
  }
  void *X = calloc((size_t)bm * bn, es), *Y = calloc((size_t)bm * bn, es);
  CHECK(dplasma_desc_get_lapack(B[0], X, bm) == 0 && dplasma_desc_get_lapack(B[1], Y, bm) == 0, "get_lapack");
  const double e = cmp_local(X, Y, cplx, bm, bn, nb, 'A');
  CHECK(e < 1e-12, "%c%s side %d uplo %d trans %d diag %d: local tiles differ by %.3e", cplx ? 'z' : 'd',
        solve ? "trsm" : "trmm", side, uplo, trans, diag, e);
  if (rank == 0)
    printf("%c%s %d/%d/%d/%d n=%d nrhs=%d grid %dx%d: max rel diff %.2e\n", cplx ? 'z' : 'd', solve ? "trsm" : "trmm",
           side, uplo, trans, diag, n, nrhs, P, Q, e);
  for (int s = 0; s < 2; ++s) dplasma_desc_destroy(A[s]), dplasma_desc_destroy(B[s]);
  free(X), free(Y);
}

/* distributed posv: the solution's local tiles equal the one-process engine's */
static void test_posv(int prec, int uplo, int n, int nrhs, int nb) {
  const int cplx = prec == dplasmaComplexDouble, es = cplx ? 16 : 8;
  dplasma_desc_t *A[2], *B[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, n, n), B[s] = mat(cx[s], prec, nb, n, nrhs);
    ok = ok && A[s] && B[s];
  }
  CHECK(ok, "descriptors");
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc = cplx ? (dplasma_zplghe(cx[s], (double)n, uplo, A[s], 31) | dplasma_zplrnt(cx[s], 0, B[s], 32))
                  : (dplasma_dplghe(cx[s], (double)n, uplo, A[s], 31) | dplasma_dplrnt(cx[s], 0, B[s], 32));
    const int info = cplx ? dplasma_zposv(cx[s], uplo, A[s], B[s]) : dplasma_dposv(cx[s], uplo, A[s], B[s]);
    CHECK(rc == 0 && info == 0, "posv (%s context): info %d %s", s ? "one-process" : "distributed", info,
          dplasma_last_error());
  }
  void *X = calloc((size_t)n * nrhs, es), *Y = calloc((size_t)n * nrhs, es);
  CHECK(dplasma_desc_get_lapack(B[0], X, n) == 0 && dplasma_desc_get_lapack(B[1], Y, n) == 0, "get_lapack");
  const double e = cmp_local(X, Y, cplx, n, nrhs, nb, 'A');
  CHECK(e < 1e-11, "%cposv uplo %d: local solution tiles differ by %.3e", cplx ? 'z' : 'd', uplo, e);
  if (rank == 0) printf("%cposv %d n=%d nrhs=%d grid %dx%d: max rel diff %.2e\n", cplx ? 'z' : 'd', uplo, n, nrhs, P, Q, e);
  for (int s = 0; s < 2; ++s) dplasma_desc_destroy(A[s]), dplasma_desc_destroy(B[s]);
  free(X), free(Y);
}

/* distributed level-3 BLAS with a symmetric / Hermitian operand or result: local tiles (of C's triangle for
 * the rank-k updates) equal the one-process engine's.  kind: 0 syrk, 1 herk, 2 syr2k, 3 her2k, 4 symm, 5 hemm */
static void test_blas3(int kind, int uplo, int trans_or_side, int n, int k, int nb) {
  const int cplx = kind == 1 || kind == 3 || kind == 5, es = cplx ? 16 : 8, prec = cplx ? dplasmaComplexDouble : dplasmaRealDouble;
  const int rank_k = kind <= 3, nt = trans_or_side == dplasmaNoTrans;
  /* rank-k: A, B are n x k (NoTrans) or k x n; symm / hemm: A n x n (side Left) or k x k, B / C n x k */
  const int am = rank_k ? (nt ? n : k) : (trans_or_side == dplasmaLeft ? n : k);
  const int an = rank_k ? (nt ? k : n) : am;
  const int cm = n, cn = rank_k ? n : k;
  dplasma_desc_t *A[2], *B[2], *C[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, am, an);
    B[s] = mat(cx[s], prec, nb, rank_k ? am : cm, rank_k ? an : cn);
    C[s] = mat(cx[s], prec, nb, cm, cn);
    ok = ok && A[s] && B[s] && C[s];
  }
  CHECK(ok, "descriptors");
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc = cplx ? (dplasma_zplrnt(cx[s], 0, A[s], 41) | dplasma_zplrnt(cx[s], 0, B[s], 42))
                  : (dplasma_dplrnt(cx[s], 0, A[s], 41) | dplasma_dplrnt(cx[s], 0, B[s], 42));
    if (kind == 1 || kind == 3) rc |= dplasma_zplghe(cx[s], 1.0, dplasmaUpperLower, C[s], 43);
    else if (cplx) rc |= dplasma_zplrnt(cx[s], 0, C[s], 43);
    else rc |= dplasma_dplrnt(cx[s], 0, C[s], 43);
    switch (kind) {
      case 0: rc |= dplasma_dsyrk(cx[s], uplo, trans_or_side, 1.25, A[s], -0.5, C[s]); break;
      case 1: rc |= dplasma_zherk(cx[s], uplo, trans_or_side, 1.25, A[s], -0.5, C[s]); break;
      case 2: rc |= dplasma_dsyr2k(cx[s], uplo, trans_or_side, 1.25, A[s], B[s], -0.5, C[s]); break;
      case 3: rc |= dplasma_zher2k(cx[s], uplo, trans_or_side, 1.25 - 0.5 * I, A[s], B[s], -0.5, C[s]); break;
      case 4: rc |= dplasma_dsymm(cx[s], trans_or_side, uplo, 1.25, A[s], B[s], -0.5, C[s]); break;
      default: rc |= dplasma_zhemm(cx[s], trans_or_side, uplo, 1.25 - 0.5 * I, A[s], B[s], -0.5 + 0.25 * I, C[s]); break;
    }
    CHECK(rc == 0, "blas3 kind %d (%s context): %s", kind, s ? "one-process" : "distributed", dplasma_last_error());
  }
  void *X = calloc((size_t)cm * cn, es), *Y = calloc((size_t)cm * cn, es);
  CHECK(dplasma_desc_get_lapack(C[0], X, cm) == 0 && dplasma_desc_get_lapack(C[1], Y, cm) == 0, "get_lapack");
  const char part = rank_k ? (uplo == dplasmaLower ? 'L' : 'U') : 'A';
  const double e = cmp_local(X, Y, cplx, cm, cn, nb, part);
  static const char *nm[6] = {"dsyrk", "zherk", "dsyr2k", "zher2k", "dsymm", "zhemm"};
  CHECK(e < 1e-12, "%s uplo %d %d: local tiles differ by %.3e", nm[kind], uplo, trans_or_side, e);
  if (rank == 0) printf("%s %d/%d n=%d k=%d grid %dx%d: max rel diff %.2e\n", nm[kind], uplo, trans_or_side, n, k, P, Q, e);
  for (int s = 0; s < 2; ++s) dplasma_desc_destroy(A[s]), dplasma_desc_destroy(B[s]), dplasma_desc_destroy(C[s]);
  free(X), free(Y);
}

/* distributed inversions: trtri (via the distributed solve on the identity), lauum (triangle product on C's
 * triangle), potri and poinv; the stored triangle's local tiles equal the one-process engine's.
 * kind: 0 trtri, 1 lauum, 2 potri (on a Cholesky factor), 3 poinv */
static void test_inv(int kind, int uplo, int diag, int n, int nb) {
  dplasma_desc_t *A[2];
  dplasma_context_t *cx[2] = {cd, c1};
  A[0] = mat(cd, dplasmaRealDouble, nb, n, n), A[1] = mat(c1, dplasmaRealDouble, nb, n, n);
  if (!A[0] || !A[1]) { CHECK(0, "descriptors"); return; }
  for (int s = 0; s < 2; ++s) {
    int rc = dplasma_dplghe(cx[s], (double)n, dplasmaUpperLower, A[s], 51);
    if (kind == 2) rc |= dplasma_dpotrf(cx[s], uplo, A[s]);
    switch (kind) {
      case 0: rc |= dplasma_dtrtri(cx[s], uplo, diag, A[s]); break;
      case 1: rc |= dplasma_dlauum(cx[s], uplo, A[s]); break;
      case 2: rc |= dplasma_dpotri(cx[s], uplo, A[s]); break;
      default: rc |= dplasma_dpoinv(cx[s], uplo, A[s]); break;
    }
    CHECK(rc == 0, "inversion kind %d (%s context): %s", kind, s ? "one-process" : "distributed", dplasma_last_error());
  }
  double *X = calloc((size_t)n * n, 8), *Y = calloc((size_t)n * n, 8);
  CHECK(dplasma_desc_get_lapack(A[0], X, n) == 0 && dplasma_desc_get_lapack(A[1], Y, n) == 0, "get_lapack");
  const double e = cmp_local(X, Y, 0, n, n, nb, uplo == dplasmaLower ? 'L' : 'U');
  static const char *nm[4] = {"dtrtri", "dlauum", "dpotri", "dpoinv"};
  CHECK(e < 1e-11, "%s uplo %d diag %d: local tiles differ by %.3e", nm[kind], uplo, diag, e);
  if (rank == 0) printf("%s %d/%d n=%d grid %dx%d: max rel diff %.2e\n", nm[kind], uplo, diag, n, P, Q, e);
  dplasma_desc_destroy(A[0]), dplasma_desc_destroy(A[1]);
  free(X), free(Y);
}

/* distributed LU with partial pivoting (getrf_1d) and gesv: the pivots (replicated) and every rank's tiles
 * of the factors / solution equal the one-process engine's */
static void test_lu(int prec, int m, int n, int nrhs, int nb) {
  const int cplx = prec == dplasmaComplexDouble, es = cplx ? 16 : 8, k = m < n ? m : n;
  dplasma_desc_t *A[2], *IP[2], *B[2] = {NULL, NULL};
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, m, n);
    IP[s] = dplasma_desc_ipiv(cx[s], 1, nb, 1, k, 1, 1);
    if (nrhs) B[s] = mat(cx[s], prec, nb, m, nrhs);
    ok = ok && A[s] && IP[s] && (!nrhs || B[s]);
  }
  CHECK(ok, "descriptors: %s", dplasma_last_error());
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc = cplx ? dplasma_zplrnt(cx[s], 0, A[s], 61) : dplasma_dplrnt(cx[s], 0, A[s], 61);
    if (nrhs) rc |= cplx ? dplasma_zplrnt(cx[s], 0, B[s], 62) : dplasma_dplrnt(cx[s], 0, B[s], 62);
    int info;
    if (nrhs) info = cplx ? dplasma_zgesv_1d(cx[s], A[s], IP[s], B[s]) : dplasma_dgesv_1d(cx[s], A[s], IP[s], B[s]);
    else info = cplx ? dplasma_zgetrf_1d(cx[s], A[s], IP[s]) : dplasma_dgetrf_1d(cx[s], A[s], IP[s]);
    CHECK(rc == 0 && info == 0, "%s (%s context): info %d %s", nrhs ? "gesv" : "getrf", s ? "one-process" : "distributed",
          info, dplasma_last_error());
  }
  int *p0 = calloc(k, sizeof(int)), *p1 = calloc(k, sizeof(int));
  CHECK(dplasma_desc_get_lapack(IP[0], p0, 1) == 0 && dplasma_desc_get_lapack(IP[1], p1, 1) == 0, "ipiv get");
  int same = 1;
  for (int i = 0; i < k; ++i) same = same && p0[i] == p1[i];
  CHECK(same, "pivots differ from one process");
  void *X = calloc((size_t)m * n, es), *Y = calloc((size_t)m * n, es);
  CHECK(dplasma_desc_get_lapack(A[0], X, m) == 0 && dplasma_desc_get_lapack(A[1], Y, m) == 0, "get_lapack");
  double e = cmp_local(X, Y, cplx, m, n, nb, 'A');
  CHECK(e < 1e-12, "%cgetrf %dx%d: local factor tiles differ by %.3e", cplx ? 'z' : 'd', m, n, e);
  if (nrhs) {
    void *U = calloc((size_t)m * nrhs, es), *V = calloc((size_t)m * nrhs, es);
    CHECK(dplasma_desc_get_lapack(B[0], U, m) == 0 && dplasma_desc_get_lapack(B[1], V, m) == 0, "get_lapack");
    const double eb = cmp_local(U, V, cplx, m, nrhs, nb, 'A');
    CHECK(eb < 1e-11, "%cgesv: local solution tiles differ by %.3e", cplx ? 'z' : 'd', eb);
    if (eb > e) e = eb;
    free(U), free(V);
  }
  if (rank == 0)
    printf("%c%s %dx%d nrhs=%d grid %dx%d: pivots %s, max rel diff %.2e\n", cplx ? 'z' : 'd', nrhs ? "gesv" : "getrf", m,
           n, nrhs, P, Q, same ? "identical" : "DIFFER", e);
  for (int s = 0; s < 2; ++s) {
    dplasma_desc_destroy(A[s]), dplasma_desc_destroy(IP[s]);
    if (B[s]) dplasma_desc_destroy(B[s]);
  }
  free(X), free(Y), free(p0), free(p1);
}

/* flat QR on the grid (geqrf, Q^H B, gels) against the one-process engine on the whole matrix: R / V
 * tiles, the T blocks' owner tile, Q^H B and the least-squares solution, each rank on its tiles */
static void test_qr(int m, int n, int nrhs, int nb, int ib) {
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A[2], *T[2], *B[2], *B2[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], dplasmaRealDouble, nb, m, n);
    B[s] = mat(cx[s], dplasmaRealDouble, nb, m, nrhs);
    B2[s] = mat(cx[s], dplasmaRealDouble, nb, m, nrhs);
    T[s] = dplasma_desc_block_cyclic(cx[s], dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 0, 0, dplasmaUpperLower);
    ok = ok && A[s] && B[s] && B2[s] && T[s];
  }
  CHECK(ok, "qr descriptors: %s", dplasma_last_error());
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc = dplasma_dplrnt(cx[s], 0, A[s], 71) | dplasma_dplrnt(cx[s], 0, B[s], 72) | dplasma_dplrnt(cx[s], 0, B2[s], 72);
    const int info = dplasma_dgeqrf(cx[s], A[s], T[s]);
    rc |= dplasma_dunmqr(cx[s], dplasmaLeft, dplasmaTrans, A[s], T[s], B[s]);
    CHECK(rc == 0 && info == 0, "geqrf / unmqr (%s context): info %d rc %d %s", s ? "one-process" : "distributed", info,
          rc, dplasma_last_error());
  }
  double *X = calloc((size_t)m * n, 8), *Y = calloc((size_t)m * n, 8);
  double *U = calloc((size_t)m * nrhs, 8), *V = calloc((size_t)m * nrhs, 8);
  CHECK(dplasma_desc_get_lapack(A[0], X, m) == 0 && dplasma_desc_get_lapack(A[1], Y, m) == 0, "get_lapack");
  const double ea = cmp_local(X, Y, 0, m, n, nb, 'A');
  CHECK(dplasma_desc_get_lapack(B[0], U, m) == 0 && dplasma_desc_get_lapack(B[1], V, m) == 0, "get_lapack");
  const double eb = cmp_local(U, V, 0, m, nrhs, nb, 'A');
  /* least squares on fresh copies */
  for (int s = 0; s < 2; ++s) {
    int rc = dplasma_dplrnt(cx[s], 0, A[s], 71);
    const int info = dplasma_dgels(cx[s], dplasmaNoTrans, A[s], T[s], B2[s]);
    CHECK(rc == 0 && info == 0, "gels (%s context): info %d %s", s ? "one-process" : "distributed", info,
          dplasma_last_error());
  }
  CHECK(dplasma_desc_get_lapack(B2[0], U, m) == 0 && dplasma_desc_get_lapack(B2[1], V, m) == 0, "get_lapack");
  const double ex = cmp_local(U, V, 0, m, nrhs, nb, 'A');
  if (rank == 0)
    printf("dgeqrf / dunmqr / dgels %dx%d nrhs=%d grid %dx%d: max rel diff R,V %.2e  Q^T B %.2e  X %.2e\n", m, n, nrhs, P, Q,
           ea, eb, ex);
  CHECK(ea < 1e-12 && eb < 1e-12 && ex < 1e-10, "distributed QR differs: %.2e %.2e %.2e", ea, eb, ex);
  for (int s = 0; s < 2; ++s)
    dplasma_desc_destroy(A[s]), dplasma_desc_destroy(T[s]), dplasma_desc_destroy(B[s]), dplasma_desc_destroy(B2[s]);
  free(X), free(Y), free(U), free(V);
}

/* tree-driven QR on the grid (geqrf_param, unmqr_param Q^H B, ungqr_param, geqrs_param; HQR greedy / greedy with
 * TS domains of a = 2 tiles over p = P process rows) against the one-process native engine with the same tree:
 * R / V tiles, Q^H B, Q and the least-squares solution, each rank on its tiles */
static void test_qr_param(int m, int n, int nrhs, int nb, int ib, int llvl, int hlvl, int a) {
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A[2], *TS[2], *TT[2], *B[2], *B2[2], *Qm[2];
  dplasma_context_t *cx[2] = {cd, c1};
  dplasma_qrtree_t qt[2];
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], dplasmaRealDouble, nb, m, n);
    B[s] = mat(cx[s], dplasmaRealDouble, nb, m, nrhs);
    B2[s] = mat(cx[s], dplasmaRealDouble, nb, m, nrhs);
    Qm[s] = mat(cx[s], dplasmaRealDouble, nb, m, n);
    TS[s] = dplasma_desc_block_cyclic(cx[s], dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 0, 0, dplasmaUpperLower);
    TT[s] = dplasma_desc_block_cyclic(cx[s], dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 0, 0, dplasmaUpperLower);
    ok = ok && A[s] && B[s] && B2[s] && Qm[s] && TS[s] && TT[s];
    memset(&qt[s], 0, sizeof qt[s]);
    if (ok) ok = dplasma_hqr_init(&qt[s], dplasmaNoTrans, A[s], llvl, hlvl, a, P, 0, 0) == 0;
  }
  CHECK(ok, "qr_param descriptors / trees: %s", dplasma_last_error());
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc = dplasma_dplrnt(cx[s], 0, A[s], 81) | dplasma_dplrnt(cx[s], 0, B[s], 82) | dplasma_dplrnt(cx[s], 0, B2[s], 82);
    const int info = dplasma_dgeqrf_param(cx[s], &qt[s], A[s], TS[s], TT[s]);
    rc |= dplasma_dunmqr_param(cx[s], dplasmaLeft, dplasmaTrans, &qt[s], A[s], TS[s], TT[s], B[s]);
    rc |= dplasma_dungqr_param(cx[s], &qt[s], A[s], TS[s], TT[s], Qm[s]);
    rc |= dplasma_dgeqrs_param(cx[s], &qt[s], A[s], TS[s], TT[s], B2[s]);
    CHECK(rc == 0 && info == 0, "geqrf_param family (%s context): info %d rc %d %s", s ? "one-process" : "distributed", info,
          rc, dplasma_last_error());
  }
  double *X = calloc((size_t)m * n, 8), *Y = calloc((size_t)m * n, 8);
  double *U = calloc((size_t)m * nrhs, 8), *V = calloc((size_t)m * nrhs, 8);
  CHECK(dplasma_desc_get_lapack(A[0], X, m) == 0 && dplasma_desc_get_lapack(A[1], Y, m) == 0, "get_lapack");
  const double ea = cmp_local(X, Y, 0, m, n, nb, 'A');
  CHECK(dplasma_desc_get_lapack(Qm[0], X, m) == 0 && dplasma_desc_get_lapack(Qm[1], Y, m) == 0, "get_lapack");
  const double eq = cmp_local(X, Y, 0, m, n, nb, 'A');
  CHECK(dplasma_desc_get_lapack(B[0], U, m) == 0 && dplasma_desc_get_lapack(B[1], V, m) == 0, "get_lapack");
  const double eb = cmp_local(U, V, 0, m, nrhs, nb, 'A');
  CHECK(dplasma_desc_get_lapack(B2[0], U, m) == 0 && dplasma_desc_get_lapack(B2[1], V, m) == 0, "get_lapack");
  const double ex = cmp_local(U, V, 0, m, nrhs, nb, 'A');
  if (rank == 0)
    printf("dgeqrf_param family %dx%d tree (%d, %d, a=%d, p=%d) grid %dx%d: max rel diff R,V %.2e  Q %.2e  Q^T B %.2e  X %.2e\n",
           m, n, llvl, hlvl, a, P, P, Q, ea, eq, eb, ex);
  CHECK(ea < 1e-12 && eq < 1e-12 && eb < 1e-12 && ex < 1e-10, "distributed tree QR differs: %.2e %.2e %.2e %.2e", ea, eq,
        eb, ex);
  for (int s = 0; s < 2; ++s) {
    dplasma_hqr_finalize(&qt[s]);
    dplasma_desc_destroy(A[s]), dplasma_desc_destroy(TS[s]), dplasma_desc_destroy(TT[s]), dplasma_desc_destroy(B[s]);
    dplasma_desc_destroy(B2[s]), dplasma_desc_destroy(Qm[s]);
  }
  free(X), free(Y), free(U), free(V);
}

/* transposed maps on the grid (a tile-by-tile distributed transpose): geadd / tradd with op(A) */
static void test_trans_maps(int cplx, int uplo, int m, int n, int nb) {
  const int prec = cplx ? dplasmaComplexDouble : dplasmaRealDouble, es = cplx ? 16 : 8;
  dplasma_desc_t *A[2], *B[2];
  dplasma_context_t *cx[2] = {cd, c1};
  int ok = 1;
  for (int s = 0; s < 2; ++s) {
    A[s] = mat(cx[s], prec, nb, n, m), B[s] = mat(cx[s], prec, nb, m, n);
    ok = ok && A[s] && B[s];
  }
  CHECK(ok, "descriptors");
  if (!ok) return;
  for (int s = 0; s < 2; ++s) {
    int rc;
    if (cplx) {
      rc = dplasma_zplrnt(cx[s], 0, A[s], 71) | dplasma_zplrnt(cx[s], 0, B[s], 72);
      rc |= dplasma_ztradd(cx[s], uplo, dplasmaConjTrans, 2.0 - 1.0 * I, A[s], -1.0, B[s]);
    } else {
      rc = dplasma_dplrnt(cx[s], 0, A[s], 71) | dplasma_dplrnt(cx[s], 0, B[s], 72);
      rc |= dplasma_dgeadd(cx[s], dplasmaTrans, 2.0, A[s], -1.0, B[s]);
    }
    CHECK(rc == 0, "transposed map (%s context): %s", s ? "one-process" : "distributed", dplasma_last_error());
  }
  void *X = calloc((size_t)m * n, es), *Y = calloc((size_t)m * n, es);
  CHECK(dplasma_desc_get_lapack(B[0], X, m) == 0 && dplasma_desc_get_lapack(B[1], Y, m) == 0, "get_lapack");
  const double e = cmp_local(X, Y, cplx, m, n, nb, 'A');
  CHECK(e == 0.0, "%s with op(A): local tiles differ by %.3e", cplx ? "ztradd" : "dgeadd", e);
  if (rank == 0) printf("%s op(A) %dx%d grid %dx%d: max rel diff %.2e\n", cplx ? "ztradd" : "dgeadd", m, n, P, Q, e);
  for (int s = 0; s < 2; ++s) dplasma_desc_destroy(A[s]), dplasma_desc_destroy(B[s]);
  free(X), free(Y);
}

static void test_failing_potrf(void) {
  /* a general random matrix is not positive definite: every rank reports the one-process info */
  const int n = 700, nb = 64;
  dplasma_desc_t *A = mat(cd, dplasmaRealDouble, nb, n, n), *B = mat(c1, dplasmaRealDouble, nb, n, n);
  CHECK(A && B, "descriptors");
  if (!A || !B) return;
  dplasma_dplrnt(cd, 0, A, 77);
  dplasma_dplrnt(c1, 0, B, 77);
  const int i1 = dplasma_dpotrf(cd, dplasmaLower, A), i2 = dplasma_dpotrf(c1, dplasmaLower, B);
  CHECK(i1 > 0 && i1 == i2, "non-SPD dpotrf info %d, one process %d", i1, i2);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

static void test_norms_maps(void) {
  const int m = 530, n = 410, nb = 64;
  dplasma_desc_t *A = mat(cd, dplasmaRealDouble, nb, m, n), *B = mat(c1, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *A2 = mat(cd, dplasmaRealDouble, nb, m, n);
  CHECK(A && B && A2, "descriptors");
  if (!A || !B || !A2) return;
  dplasma_dplrnt(cd, 0, A, 5);
  dplasma_dplrnt(c1, 0, B, 5);
  {
    /* host view: this rank's tiles of A against the one-process matrix */
    double *X = calloc((size_t)m * n, 8), *Y = calloc((size_t)m * n, 8);
    dplasma_desc_get_lapack(A, X, m);
    dplasma_desc_get_lapack(B, Y, m);
    const double e = cmp_local(X, Y, 0, m, n, nb, 'A');
    double lx = 0, ly = 0;
    int ix = -1, iy = -1;
    for (int i = 0; i < m * n; ++i) {
      if (fabs(Y[i]) > ly) ly = fabs(Y[i]), iy = i;
      if (((i % m) / nb) % P == rank / Q && ((i / m) / nb) % Q == rank % Q && fabs(X[i]) > lx) lx = fabs(X[i]), ix = i;
    }
    CHECK(e == 0, "plrnt: local tiles differ from one process by %.3e", e);
    printf("rank %d: local max %.15g at (%d,%d); one-process max %.15g at (%d,%d)\n", rank, lx, ix % m, ix / m, ly,
           iy % m, iy / m);
    free(X), free(Y);
  }
  const int nt[4] = {dplasmaMaxNorm, dplasmaOneNorm, dplasmaInfNorm, dplasmaFrobeniusNorm};
  for (int t = 0; t < 4; ++t) {
    const double x = dplasma_dlange(cd, nt[t], A), y = dplasma_dlange(c1, nt[t], B);
    CHECK(fabs(x - y) <= 1e-12 * y, "dlange %d: %.15g vs one process %.15g", nt[t], x, y);
  }
  /* A2 = A; A2 = 2 A2 - A = A; lower part zeroed with diagonal 3: lange max == max(3, max |upper|) */
  CHECK(dplasma_dlacpy(cd, dplasmaUpperLower, A, A2) == 0, "dlacpy: %s", dplasma_last_error());
  {
    double *X = calloc((size_t)m * n, 8), *Y = calloc((size_t)m * n, 8);
    dplasma_desc_get_lapack(A, X, m);
    dplasma_desc_get_lapack(A2, Y, m);
    const double e = cmp_local(Y, X, 0, m, n, nb, 'A');
    CHECK(e == 0, "lacpy: local tiles differ from A by %.3e", e);
    free(X), free(Y);
  }
  CHECK(dplasma_dgeadd(cd, dplasmaNoTrans, -1.0, A, 2.0, A2) == 0, "dgeadd: %s", dplasma_last_error());
  const double d = dplasma_dlange(cd, dplasmaFrobeniusNorm, A2), a = dplasma_dlange(cd, dplasmaFrobeniusNorm, A);
  CHECK(fabs(d - a) <= 1e-12 * a, "lacpy + geadd: |A2|_F %.15g vs |A|_F %.15g", d, a);
  {   /* symmetric / Hermitian norms of a square matrix's triangle (mirror exchange + all-reduced partials) */
    const int ns = 450, nbs = 64;
    dplasma_desc_t *S0 = mat(cd, dplasmaRealDouble, nbs, ns, ns), *S1 = mat(c1, dplasmaRealDouble, nbs, ns, ns);
    dplasma_desc_t *Z0 = mat(cd, dplasmaComplexDouble, nbs, ns, ns), *Z1 = mat(c1, dplasmaComplexDouble, nbs, ns, ns);
    if (S0 && S1 && Z0 && Z1) {
      dplasma_dplrnt(cd, 0, S0, 9), dplasma_dplrnt(c1, 0, S1, 9);
      dplasma_zplrnt(cd, 0, Z0, 9), dplasma_zplrnt(c1, 0, Z1, 9);
      for (int t = 0; t < 4; ++t)
        for (int u = 0; u < 2; ++u) {
          const int up = u ? dplasmaUpper : dplasmaLower;
          const double x = dplasma_dlansy(cd, nt[t], up, S0), y = dplasma_dlansy(c1, nt[t], up, S1);
          CHECK(fabs(x - y) <= 1e-12 * y, "dlansy %d %d: %.15g vs one process %.15g", nt[t], up, x, y);
          const double zx = dplasma_zlanhe(cd, nt[t], up, Z0), zy = dplasma_zlanhe(c1, nt[t], up, Z1);
          CHECK(fabs(zx - zy) <= 1e-12 * zy, "zlanhe %d %d: %.15g vs one process %.15g", nt[t], up, zx, zy);
        }
    } else {
      CHECK(0, "descriptors");
    }
    dplasma_desc_destroy(S0), dplasma_desc_destroy(S1), dplasma_desc_destroy(Z0), dplasma_desc_destroy(Z1);
  }
  CHECK(dplasma_dlaset(cd, dplasmaLower, 0.0, 3.0, A2) == 0, "dlaset: %s", dplasma_last_error());
  CHECK(dplasma_dlaset(c1, dplasmaLower, 0.0, 3.0, B) == 0, "dlaset (one process)");
  const double l1 = dplasma_dlange(cd, dplasmaOneNorm, A2), l2 = dplasma_dlange(c1, dplasmaOneNorm, B);
  CHECK(fabs(l1 - l2) <= 1e-12 * l2, "laset + lange one: %.15g vs %.15g", l1, l2);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(A2);
}

static void test_taskpool_and_refusal(void) {
  const int n = 512, nb = 128;
  dplasma_desc_t *A = mat(cd, dplasmaRealDouble, nb, n, n), *B = mat(cd, dplasmaRealDouble, nb, n, n);
  if (!A || !B) { CHECK(0, "descriptors"); return; }
  dplasma_dplghe(cd, (double)n, dplasmaLower, A, 1);
  dplasma_taskpool_t *tp = dplasma_dpotrf_New(cd, dplasmaLower, A);
  CHECK(tp != NULL, "dpotrf_New: %s", dplasma_last_error());
  if (tp) {
    CHECK(dplasma_context_add_taskpool(cd, tp) == 0 && dplasma_context_start(cd) == 0 && dplasma_context_wait(cd) == 0,
          "taskpool lifecycle");
    CHECK(dplasma_taskpool_result(tp) == 0, "taskpool info %d", dplasma_taskpool_result(tp));
    dplasma_dpotrf_Destruct(tp);
  }
  /* no distributed LQ builder: a clean error on every rank, the context stays usable */
  const int rc = dplasma_dgelqf(cd, A, B);
  CHECK(rc != 0 && strstr(dplasma_last_error(), "multi-process"), "dgelqf on a multi-process context: rc %d '%s'", rc,
        dplasma_last_error());
  CHECK(dplasma_dlange(cd, dplasmaMaxNorm, A) > 0, "context usable after a refused call");
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

int main(int argc, char **argv) {
  if (argc < 5) {
    printf("usage: test_native_dist rank world P rdv_dir\n");
    return 2;
  }
  rank = atoi(argv[1]), world = atoi(argv[2]), P = atoi(argv[3]);
  Q = world / P;
  cd = dplasma_init_native_dist(0, rank, world, P, argv[4]);
  c1 = dplasma_init_native(0);
  if (!cd || !c1) {
    printf("rank %d: init failed: %s\n", rank, dplasma_last_error());
    return 2;
  }
  CHECK(dplasma_context_rank(cd) == rank && dplasma_context_world(cd) == world, "rank / world of the context");
  setvbuf(stdout, NULL, _IOLBF, 0);
  printf("rank %d: contexts up\n", rank);
  test_potrf(dplasmaRealDouble, 'L', 1100, 128);
  test_potrf(dplasmaRealDouble, 'U', 1100, 128);
  test_potrf(dplasmaRealDouble, 'L', 2048, 256);
  test_potrf(dplasmaComplexDouble, 'L', 600, 96);
  test_potrf(dplasmaComplexDouble, 'U', 600, 96);
  test_gemm(dplasmaRealDouble, dplasmaNoTrans, dplasmaNoTrans, 700, 500, 900, 128);
  test_gemm(dplasmaRealDouble, dplasmaTrans, dplasmaNoTrans, 640, 384, 520, 128);
  test_gemm(dplasmaRealDouble, dplasmaNoTrans, dplasmaTrans, 300, 700, 257, 64);
  test_gemm(dplasmaComplexDouble, dplasmaConjTrans, dplasmaTrans, 260, 330, 190, 64);
  test_trxm(dplasmaRealDouble, 1, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, 700, 300, 128);
  test_trxm(dplasmaRealDouble, 1, dplasmaLeft, dplasmaUpper, dplasmaTrans, dplasmaUnit, 700, 300, 128);
  test_trxm(dplasmaRealDouble, 1, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 520, 200, 64);
  test_trxm(dplasmaRealDouble, 1, dplasmaRight, dplasmaLower, dplasmaTrans, dplasmaNonUnit, 520, 330, 64);
  test_trxm(dplasmaRealDouble, 1, dplasmaRight, dplasmaUpper, dplasmaNoTrans, dplasmaUnit, 520, 330, 64);
  test_trxm(dplasmaComplexDouble, 1, dplasmaLeft, dplasmaLower, dplasmaConjTrans, dplasmaNonUnit, 300, 170, 64);
  test_trxm(dplasmaComplexDouble, 1, dplasmaRight, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, 300, 170, 64);
  test_trxm(dplasmaRealDouble, 0, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaUnit, 600, 250, 128);
  test_trxm(dplasmaRealDouble, 0, dplasmaRight, dplasmaUpper, dplasmaTrans, dplasmaNonUnit, 520, 330, 64);
  test_blas3(0, dplasmaLower, dplasmaNoTrans, 530, 300, 64);
  test_blas3(0, dplasmaUpper, dplasmaTrans, 530, 300, 64);
  test_blas3(1, dplasmaLower, dplasmaConjTrans, 330, 200, 64);
  test_blas3(2, dplasmaUpper, dplasmaNoTrans, 400, 270, 64);
  test_blas3(3, dplasmaLower, dplasmaNoTrans, 330, 200, 64);
  test_blas3(4, dplasmaLower, dplasmaLeft, 450, 310, 64);
  test_blas3(4, dplasmaUpper, dplasmaRight, 450, 310, 64);
  test_blas3(5, dplasmaUpper, dplasmaLeft, 300, 170, 64);
  test_inv(0, dplasmaLower, dplasmaNonUnit, 520, 64);
  test_inv(0, dplasmaUpper, dplasmaUnit, 520, 64);
  test_inv(1, dplasmaLower, dplasmaNonUnit, 450, 64);
  test_inv(1, dplasmaUpper, dplasmaNonUnit, 450, 64);
  test_inv(2, dplasmaLower, dplasmaNonUnit, 450, 64);
  test_inv(3, dplasmaUpper, dplasmaNonUnit, 450, 64);
  test_lu(dplasmaRealDouble, 600, 600, 0, 64);
  test_lu(dplasmaRealDouble, 700, 500, 0, 64);
  test_lu(dplasmaRealDouble, 400, 600, 0, 64);
  test_lu(dplasmaRealDouble, 640, 640, 90, 128);
  test_lu(dplasmaComplexDouble, 300, 300, 40, 64);
  test_posv(dplasmaRealDouble, dplasmaLower, 900, 130, 128);
  test_posv(dplasmaRealDouble, dplasmaUpper, 900, 130, 128);
  test_posv(dplasmaComplexDouble, dplasmaLower, 400, 70, 64);
  test_qr(700, 450, 30, 64, 16);
  test_qr(512, 512, 64, 128, 32);
  test_qr_param(700, 450, 30, 64, 16, 1, 1, 2);
  test_qr_param(520, 520, 20, 64, 16, 3, 0, 1);
  test_trans_maps(0, dplasmaUpperLower, 530, 410, 64);
  test_trans_maps(1, dplasmaLower, 330, 330, 64);
  test_failing_potrf();
  test_norms_maps();
  test_taskpool_and_refusal();
  CHECK(!dplasma_python_active(), "the embedded interpreter was started");
  dplasma_fini(c1);
  dplasma_fini(cd);
  if (fails) {
    printf("rank %d: native dist: %d FAILED\n", rank, fails);
    return 1;
  }
  printf("rank %d: native dist: all passed\n", rank);
  return 0;
}
