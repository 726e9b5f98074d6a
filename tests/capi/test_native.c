/* Interpreter-free C ABI (dplasma_init_native, capi/native.cpp) on one GPU: Cholesky / solve / GEMM /
 * TRSM against host reference arithmetic, the taskpool lifecycle, an unsupported call, and a
 * check that the embedded interpreter was never started.
 * usage: test_native [N_bench]   (N_bench > 0: also time dpotrf at N_bench, NB = 512) */
#include <complex.h>
#include <execinfo.h>
#include <math.h>
#include <signal.h>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dplasma.h"

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      printf("FAIL %s:%d ", __FILE__, __LINE__); \
      printf(__VA_ARGS__);                    \
      printf("\n");                           \
      fails++;                                \
    }                                         \
  } while (0)

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static dplasma_desc_t *dmat(dplasma_context_t *ctx, int prec, int nb, int m, int n) {
  dplasma_desc_t *A = dplasma_desc_block_cyclic(ctx, prec, nb, nb, m, n, 1, 1, dplasmaUpperLower);
  if (!A) printf("desc: %s\n", dplasma_last_error());
  return A;
}

/* ||A0 - L L^T||_max / (n ||A0||_max) on the lower triangle (A0 lower holds the input) */
static double chol_resid_d(const double *A0, const double *L, int n) {
  double err = 0, nrm = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += L[i + (size_t)k * n] * L[j + (size_t)k * n];
      err = fmax(err, fabs(A0[i + (size_t)j * n] - s));
      nrm = fmax(nrm, fabs(A0[i + (size_t)j * n]));
    }
  return err / (n * nrm);
}

static void test_dpotrf_posv(dplasma_context_t *ctx) {
  const int n = 1200, nb = 256, nrhs = 70;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  dplasma_desc_t *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  double *A0 = malloc(sizeof(double) * n * n), *L = malloc(sizeof(double) * n * n);
  double *B0 = malloc(sizeof(double) * n * nrhs), *X = malloc(sizeof(double) * n * nrhs);
  CHECK(A && B, "descriptors");
  CHECK(dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 3872) == 0, "dplghe: %s", dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, A0, n) == 0, "get A0");
  int info = dplasma_dpotrf(ctx, dplasmaLower, A);
  CHECK(info == 0, "dpotrf info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, L, n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < j; ++i) L[i + (size_t)j * n] = 0.0;
  const double r = chol_resid_d(A0, L, n);
  printf("dpotrf n=%d nb=%d residual %.3e\n", n, nb, r);
  CHECK(r < 1e-14, "dpotrf residual %.3e", r);

  /* posv on a fresh copy of A: A0 x = b */
  CHECK(dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 3872) == 0, "dplghe 2");
  CHECK(dplasma_dplrnt(ctx, 0, B, 51) == 0, "dplrnt: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, B0, n);
  info = dplasma_dposv(ctx, dplasmaLower, A, B);
  CHECK(info == 0, "dposv info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(B, X, n);
  double err = 0, bn = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) {
        const double a = i >= k ? A0[i + (size_t)k * n] : A0[k + (size_t)i * n];
        s += a * X[k + (size_t)c * n];
      }
      err = fmax(err, fabs(s - B0[i + (size_t)c * n]));
      bn = fmax(bn, fabs(B0[i + (size_t)c * n]));
    }
  printf("dposv n=%d nrhs=%d ||Ax-b||/||b|| %.3e\n", n, nrhs, err / bn);
  CHECK(err / bn < 1e-12, "dposv residual %.3e", err / bn);
  free(A0), free(L), free(B0), free(X);
  dplasma_desc_destroy(A);
  dplasma_desc_destroy(B);
}

/* posv on a single tile (n <= nb): the solves must wait for the tile factorisation (one POTRF and two
 * TRSM tasks on different streams) */
static void test_dposv_one_tile(dplasma_context_t *ctx) {
  const int n = 200, nb = 256, nrhs = 9;
  for (int rep = 0; rep < 3; ++rep) {
    dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
    double *A0 = malloc(sizeof(double) * n * n), *B0 = malloc(sizeof(double) * n * nrhs);
    double *X = malloc(sizeof(double) * n * nrhs);
    dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 11 + rep);
    dplasma_dplrnt(ctx, 0, B, 12 + rep);
    dplasma_desc_get_lapack(A, A0, n);
    dplasma_desc_get_lapack(B, B0, n);
    const int info = dplasma_dposv(ctx, dplasmaLower, A, B);
    CHECK(info == 0, "dposv (one tile) info %d (%s)", info, dplasma_last_error());
    dplasma_desc_get_lapack(B, X, n);
    double err = 0, bn = 0;
    for (int c = 0; c < nrhs; ++c)
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += (i >= k ? A0[i + (size_t)k * n] : A0[k + (size_t)i * n]) * X[k + (size_t)c * n];
        err = fmax(err, fabs(s - B0[i + (size_t)c * n]));
        bn = fmax(bn, fabs(B0[i + (size_t)c * n]));
      }
    if (rep == 0) printf("dposv one tile n=%d nb=%d ||Ax-b||/||b|| %.3e\n", n, nb, err / bn);
    CHECK(err / bn < 1e-12, "dposv (one tile) residual %.3e", err / bn);
    free(A0), free(B0), free(X);
    dplasma_desc_destroy(A), dplasma_desc_destroy(B);
  }
}

static void test_dgemm(dplasma_context_t *ctx) {
  const int M = 300, N = 200, K = 250, nb = 128;
  /* C = alpha A^T B + beta C, A is K x M */
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, K, M), *B = dmat(ctx, dplasmaRealDouble, nb, K, N);
  dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, M, N);
  dplasma_dplrnt(ctx, 0, A, 1);
  dplasma_dplrnt(ctx, 0, B, 2);
  dplasma_dplrnt(ctx, 0, C, 3);
  double *a = malloc(sizeof(double) * K * M), *b = malloc(sizeof(double) * K * N), *c = malloc(sizeof(double) * M * N);
  double *r = malloc(sizeof(double) * M * N);
  dplasma_desc_get_lapack(A, a, K);
  dplasma_desc_get_lapack(B, b, K);
  dplasma_desc_get_lapack(C, c, M);
  const double alpha = 1.5, beta = -0.5;
  CHECK(dplasma_dgemm(ctx, dplasmaTrans, dplasmaNoTrans, alpha, A, B, beta, C) == 0, "dgemm: %s",
        dplasma_last_error());
  dplasma_desc_get_lapack(C, r, M);
  double err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      for (int k = 0; k < K; ++k) s += a[k + (size_t)i * K] * b[k + (size_t)j * K];
      err = fmax(err, fabs(alpha * s + beta * c[i + (size_t)j * M] - r[i + (size_t)j * M]));
    }
  printf("dgemm TN %dx%dx%d max error %.3e\n", M, N, K, err);
  CHECK(err < 1e-12, "dgemm error %.3e", err);
  free(a), free(b), free(c), free(r);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(C);
}

/* dsyrk (lower, A^T A) and zherk (upper, A A^H) against host sums; ragged 300 / 200 with nb 128 */
static void test_rank_k(dplasma_context_t *ctx) {
  const int N = 300, K = 200, nb = 128;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, K, N), *C = dmat(ctx, dplasmaRealDouble, nb, N, N);
  dplasma_dplrnt(ctx, 0, A, 7);
  dplasma_dplrnt(ctx, 0, C, 8);
  double *a = malloc(sizeof(double) * K * N), *c = malloc(sizeof(double) * N * N), *r = malloc(sizeof(double) * N * N);
  dplasma_desc_get_lapack(A, a, K);
  dplasma_desc_get_lapack(C, c, N);
  CHECK(dplasma_dsyrk(ctx, dplasmaLower, dplasmaTrans, 0.5, A, 2.0, C) == 0, "dsyrk: %s", dplasma_last_error());
  dplasma_desc_get_lapack(C, r, N);
  double err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double ref = c[i + (size_t)j * N];
      if (i >= j) {
        double s = 0;
        for (int k = 0; k < K; ++k) s += a[k + (size_t)i * K] * a[k + (size_t)j * K];
        ref = 0.5 * s + 2.0 * ref;
      }
      err = fmax(err, fabs(ref - r[i + (size_t)j * N]));   /* the upper part must be untouched */
    }
  printf("dsyrk LT %dx%d max error %.3e\n", N, K, err);
  CHECK(err < 1e-12, "dsyrk error %.3e", err);
  free(a), free(c), free(r);
  dplasma_desc_destroy(A), dplasma_desc_destroy(C);

  dplasma_desc_t *Z = dmat(ctx, dplasmaComplexDouble, nb, N, K), *W = dmat(ctx, dplasmaComplexDouble, nb, N, N);
  dplasma_zplrnt(ctx, 0, Z, 9);
  dplasma_zplghe(ctx, 0.0, dplasmaUpperLower, W, 10);
  double complex *z = malloc(sizeof(double complex) * N * K), *w = malloc(sizeof(double complex) * N * N);
  double complex *q = malloc(sizeof(double complex) * N * N);
  dplasma_desc_get_lapack(Z, z, N);
  dplasma_desc_get_lapack(W, w, N);
  CHECK(dplasma_zherk(ctx, dplasmaUpper, dplasmaNoTrans, -1.0, Z, 0.5, W) == 0, "zherk: %s", dplasma_last_error());
  dplasma_desc_get_lapack(W, q, N);
  err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i <= j; ++i) {
      double complex s = 0;
      for (int k = 0; k < K; ++k) s += z[i + (size_t)k * N] * conj(z[j + (size_t)k * N]);
      err = fmax(err, cabs(-s + 0.5 * w[i + (size_t)j * N] - q[i + (size_t)j * N]));
    }
  printf("zherk UN %dx%d max error %.3e\n", N, K, err);
  CHECK(err < 1e-11, "zherk error %.3e", err);
  for (int i = 0; i < N; ++i)   /* Hermitian rank-k: a real diagonal, exactly */
    CHECK(cimag(q[i + (size_t)i * N]) == 0.0, "zherk diagonal (%d) imaginary part %.3e", i, cimag(q[i + (size_t)i * N]));
  free(z), free(w), free(q);
  dplasma_desc_destroy(Z), dplasma_desc_destroy(W);
}

/* element-wise maps: dgeadd (B = 2 A^T - B), dtradd (lower), dlacpy (upper), dlaset (lower), dlascal */
static void test_maps(dplasma_context_t *ctx) {
  const int M = 260, N = 190, nb = 64;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, N, M), *B = dmat(ctx, dplasmaRealDouble, nb, M, N);
  dplasma_desc_t *S = dmat(ctx, dplasmaRealDouble, nb, M, M), *T = dmat(ctx, dplasmaRealDouble, nb, M, M);
  dplasma_dplrnt(ctx, 0, A, 21);
  dplasma_dplrnt(ctx, 0, B, 22);
  dplasma_dplrnt(ctx, 0, S, 23);
  dplasma_dplrnt(ctx, 0, T, 24);
  double *a = malloc(sizeof(double) * N * M), *b = malloc(sizeof(double) * M * N), *r = malloc(sizeof(double) * M * N);
  double *s0 = malloc(sizeof(double) * M * M), *t0 = malloc(sizeof(double) * M * M), *t1 = malloc(sizeof(double) * M * M);
  dplasma_desc_get_lapack(A, a, N);
  dplasma_desc_get_lapack(B, b, M);
  dplasma_desc_get_lapack(S, s0, M);
  dplasma_desc_get_lapack(T, t0, M);
  CHECK(dplasma_dgeadd(ctx, dplasmaTrans, 2.0, A, -1.0, B) == 0, "dgeadd: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, r, M);
  double err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) err = fmax(err, fabs(2.0 * a[j + (size_t)i * N] - b[i + (size_t)j * M] - r[i + (size_t)j * M]));
  CHECK(err < 1e-14, "dgeadd error %.3e", err);
  /* T := S on the upper triangle (lacpy), T := 3 S + T on the lower (tradd), T := -2 T (lascal) */
  CHECK(dplasma_dlacpy(ctx, dplasmaUpper, S, T) == 0, "dlacpy: %s", dplasma_last_error());
  CHECK(dplasma_dtradd(ctx, dplasmaLower, dplasmaNoTrans, 3.0, S, 1.0, T) == 0, "dtradd: %s", dplasma_last_error());
  CHECK(dplasma_dlascal(ctx, dplasmaUpperLower, -2.0, T) == 0, "dlascal: %s", dplasma_last_error());
  dplasma_desc_get_lapack(T, t1, M);
  err = 0;
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < M; ++i) {
      const double sv = s0[i + (size_t)j * M], tv = t0[i + (size_t)j * M];
      double ref = i < j ? sv : (i == j ? sv + 3.0 * sv : tv + 3.0 * sv);
      err = fmax(err, fabs(-2.0 * ref - t1[i + (size_t)j * M]));
    }
  CHECK(err < 1e-13, "lacpy/tradd/lascal error %.3e", err);
  CHECK(dplasma_dlaset(ctx, dplasmaLower, 0.25, 4.0, T) == 0, "dlaset: %s", dplasma_last_error());
  dplasma_desc_get_lapack(T, t0, M);
  err = 0;
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < M; ++i) {
      const double ref = i > j ? 0.25 : (i == j ? 4.0 : t1[i + (size_t)j * M]);
      err = fmax(err, fabs(ref - t0[i + (size_t)j * M]));
    }
  CHECK(err == 0, "dlaset error %.3e", err);
  printf("native maps (geadd, lacpy, tradd, lascal, laset) ok\n");
  free(a), free(b), free(r), free(s0), free(t0), free(t1);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(S), dplasma_desc_destroy(T);
}

/* dlange (max / one / inf / Frobenius) and zlantr (lower, unit) against host loops; ragged tiles */
static void test_norms(dplasma_context_t *ctx) {
  const int M = 300, N = 170, nb = 64;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, M, N);
  dplasma_dplrnt(ctx, 0, A, 31);
  double *a = malloc(sizeof(double) * M * N);
  dplasma_desc_get_lapack(A, a, M);
  double mx = 0, one = 0, inf = 0, fr = 0;
  double *rs = calloc(M, sizeof(double));
  for (int j = 0; j < N; ++j) {
    double cs = 0;
    for (int i = 0; i < M; ++i) {
      const double v = fabs(a[i + (size_t)j * M]);
      mx = fmax(mx, v), cs += v, rs[i] += v, fr += v * v;
    }
    one = fmax(one, cs);
  }
  for (int i = 0; i < M; ++i) inf = fmax(inf, rs[i]);
  fr = sqrt(fr);
  const double g[4] = {dplasma_dlange(ctx, dplasmaMaxNorm, A), dplasma_dlange(ctx, dplasmaOneNorm, A),
                       dplasma_dlange(ctx, dplasmaInfNorm, A), dplasma_dlange(ctx, dplasmaFrobeniusNorm, A)};
  const double r[4] = {mx, one, inf, fr};
  for (int q = 0; q < 4; ++q) CHECK(fabs(g[q] - r[q]) <= 1e-13 * r[q], "dlange kind %d: %.15e vs %.15e", q, g[q], r[q]);
  free(a), free(rs);
  dplasma_desc_destroy(A);

  dplasma_desc_t *Z = dmat(ctx, dplasmaComplexDouble, nb, N, N);
  dplasma_zplrnt(ctx, 0, Z, 32);
  double complex *z = malloc(sizeof(double complex) * N * N);
  dplasma_desc_get_lapack(Z, z, N);
  double one_z = 0;
  for (int j = 0; j < N; ++j) {
    double cs = 1.0;   /* unit diagonal */
    for (int i = j + 1; i < N; ++i) cs += cabs(z[i + (size_t)j * N]);
    one_z = fmax(one_z, cs);
  }
  const double gz = dplasma_zlantr(ctx, dplasmaOneNorm, dplasmaLower, dplasmaUnit, Z);
  CHECK(fabs(gz - one_z) <= 1e-13 * one_z, "zlantr one: %.15e vs %.15e", gz, one_z);
  printf("native norms (dlange max/one/inf/frb, zlantr) ok\n");
  /* dplgsy == dplghe for a real matrix (same LCG stream, same bump on the diagonal) */
  dplasma_desc_t *G1 = dmat(ctx, dplasmaRealDouble, nb, 150, 150), *G2 = dmat(ctx, dplasmaRealDouble, nb, 150, 150);
  CHECK(dplasma_dplgsy(ctx, 7.0, dplasmaUpperLower, G1, 41) == 0, "dplgsy: %s", dplasma_last_error());
  CHECK(dplasma_dplghe(ctx, 7.0, dplasmaUpperLower, G2, 41) == 0, "dplghe: %s", dplasma_last_error());
  double *g1 = malloc(sizeof(double) * 150 * 150), *g2 = malloc(sizeof(double) * 150 * 150);
  dplasma_desc_get_lapack(G1, g1, 150);
  dplasma_desc_get_lapack(G2, g2, 150);
  CHECK(memcmp(g1, g2, sizeof(double) * 150 * 150) == 0, "dplgsy differs from dplghe");
  free(g1), free(g2);
  dplasma_desc_destroy(G1), dplasma_desc_destroy(G2);
  free(z);
  dplasma_desc_destroy(Z);
}

/* op(T) X = alpha B (left) / X op(T) = alpha B (right) for the given variant; T = plghe (well conditioned) */
static void test_dtrsm(dplasma_context_t *ctx, int side, int uplo, int trans) {
  const int n = 400, nrhs = 150, nb = 128;
  const int bm = side == dplasmaLeft ? n : nrhs, bn = side == dplasmaLeft ? nrhs : n;
  dplasma_desc_t *T = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, bm, bn);
  dplasma_dplghe(ctx, (double)n, dplasmaUpperLower, T, 7);
  dplasma_dplrnt(ctx, 0, B, 8);
  double *t = malloc(sizeof(double) * n * n), *b0 = malloc(sizeof(double) * bm * bn), *x = malloc(sizeof(double) * bm * bn);
  dplasma_desc_get_lapack(T, t, n);
  dplasma_desc_get_lapack(B, b0, bm);
  const double alpha = 2.0;
  CHECK(dplasma_dtrsm(ctx, side, uplo, trans, dplasmaNonUnit, alpha, T, B) == 0, "dtrsm: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, x, bm);
  /* op(T) element (i, k) of the triangle */
#define TR(i, k) (((uplo == dplasmaLower) ? ((i) >= (k)) : ((i) <= (k))) ? t[(i) + (size_t)(k) * n] : 0.0)
#define OPT(i, k) (trans == dplasmaNoTrans ? TR(i, k) : TR(k, i))
  double err = 0;
  for (int j = 0; j < bn; ++j)
    for (int i = 0; i < bm; ++i) {
      double s = 0;
      if (side == dplasmaLeft)
        for (int k = 0; k < n; ++k) s += OPT(i, k) * x[k + (size_t)j * bm];
      else
        for (int k = 0; k < n; ++k) s += x[i + (size_t)k * bm] * OPT(k, j);
      err = fmax(err, fabs(s - alpha * b0[i + (size_t)j * bm]));
    }
#undef OPT
#undef TR
  printf("dtrsm side=%d uplo=%d trans=%d residual %.3e\n", side, uplo, trans, err);
  CHECK(err < 1e-10, "dtrsm residual %.3e", err);
  free(t), free(b0), free(x);
  dplasma_desc_destroy(T), dplasma_desc_destroy(B);
}

static void test_zpotrf_spotrf(dplasma_context_t *ctx) {
  /* tiles wider than the 128-wide sub-steps of the non-fp64 diagonal tiles, ragged edges */
  int n = 700, nb = 300;
  dplasma_desc_t *A = dmat(ctx, dplasmaComplexDouble, nb, n, n);
  double complex *A0 = malloc(sizeof(double complex) * n * n), *L = malloc(sizeof(double complex) * n * n);
  CHECK(dplasma_zplghe(ctx, (double)n, dplasmaLower, A, 11) == 0, "zplghe: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, A0, n);
  int info = dplasma_zpotrf(ctx, dplasmaLower, A);
  CHECK(info == 0, "zpotrf info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, L, n);
  double err = 0, nrm = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) {
      double complex s = 0;
      for (int k = 0; k <= j; ++k) s += L[i + (size_t)k * n] * conj(L[j + (size_t)k * n]);
      err = fmax(err, cabs(A0[i + (size_t)j * n] - s));
      nrm = fmax(nrm, cabs(A0[i + (size_t)j * n]));
    }
  printf("zpotrf n=%d residual %.3e\n", n, err / (n * nrm));
  CHECK(err / (n * nrm) < 1e-14, "zpotrf residual");
  free(A0), free(L);
  dplasma_desc_destroy(A);

  n = 600, nb = 256;
  dplasma_desc_t *S = dmat(ctx, dplasmaRealFloat, nb, n, n);
  float *s0 = malloc(sizeof(float) * n * n), *sl = malloc(sizeof(float) * n * n);
  dplasma_splghe(ctx, (double)n, dplasmaUpper, S, 12);
  dplasma_desc_get_lapack(S, s0, n);
  info = dplasma_spotrf(ctx, dplasmaUpper, S);
  CHECK(info == 0, "spotrf info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(S, sl, n);
  err = 0, nrm = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i <= j; ++i) {   /* A = U^T U on the upper triangle */
      double s = 0;
      for (int k = 0; k <= i; ++k) s += (double)sl[k + (size_t)i * n] * sl[k + (size_t)j * n];
      err = fmax(err, fabs(s0[i + (size_t)j * n] - s));
      nrm = fmax(nrm, fabs(s0[i + (size_t)j * n]));
    }
  printf("spotrf upper n=%d residual %.3e\n", n, err / (n * nrm));
  CHECK(err / (n * nrm) < 1e-6, "spotrf residual");
  free(s0), free(sl);
  dplasma_desc_destroy(S);
}

static void test_taskpools(dplasma_context_t *ctx) {
  const int n = 1024, nb = 256;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, n);
  dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 5);
  dplasma_dplghe(ctx, (double)n, dplasmaLower, B, 5);
  /* make B indefinite at column 700: info = 701 */
  double *h = malloc(sizeof(double) * n * n);
  dplasma_desc_get_lapack(B, h, n);
  h[700 + (size_t)700 * n] = -1.0e6;
  dplasma_desc_set_lapack(B, h, n);
  dplasma_taskpool_t *t1 = dplasma_dpotrf_New(ctx, dplasmaLower, A), *t2 = dplasma_dpotrf_New(ctx, dplasmaLower, B);
  CHECK(t1 && t2, "dpotrf_New: %s", dplasma_last_error());
  dplasma_context_add_taskpool(ctx, t1);
  dplasma_context_add_taskpool(ctx, t2);
  CHECK(dplasma_context_start(ctx) == 0, "start");
  CHECK(dplasma_context_wait(ctx) == 0, "wait");
  CHECK(dplasma_taskpool_result(t1) == 0, "t1 info %d", dplasma_taskpool_result(t1));
  CHECK(dplasma_taskpool_result(t2) == 701, "t2 info %d (expected 701)", dplasma_taskpool_result(t2));
  printf("taskpools: info %d, %d\n", dplasma_taskpool_result(t1), dplasma_taskpool_result(t2));
  /* re-run a built taskpool on a fresh matrix */
  dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 5);
  dplasma_context_add_taskpool(ctx, t1);
  dplasma_context_wait(ctx);
  CHECK(dplasma_taskpool_result(t1) == 0, "t1 rerun");
  dplasma_dpotrf_Destruct(t1);
  dplasma_dpotrf_Destruct(t2);
  free(h);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

static void bench(dplasma_context_t *ctx, int n) {
  const int nb = 512;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  dplasma_desc_t *A0 = dmat(ctx, dplasmaRealDouble, nb, n, n);
  dplasma_dplghe(ctx, (double)n, dplasmaLower, A0, 3872);
  dplasma_taskpool_t *tp = dplasma_dpotrf_New(ctx, dplasmaLower, A);
  const double fl = (double)n * n * n / 3.0 + (double)n * n / 2.0 + n / 6.0;
  for (int r = 0; r < 4; ++r) {
    dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 3872);
    const double t0 = now();
    dplasma_context_add_taskpool(ctx, tp);
    dplasma_context_wait(ctx);
    const double t = now() - t0;
    printf("[****] TIME(s) %12.5f : dpotrf native N= %d NB= %d : %14.3f gflops info=%d\n", t, n, nb, fl / t / 1e9,
           dplasma_taskpool_result(tp));
  }
  dplasma_dpotrf_Destruct(tp);
  dplasma_desc_destroy(A), dplasma_desc_destroy(A0);
}

static void on_fault(int sig) {
  void *fr[64];
  const int n = backtrace(fr, 64);
  dprintf(2, "fatal signal %d, backtrace:\n", sig);
  backtrace_symbols_fd(fr, n, 2);
  _exit(128 + sig);
}

/* dense host reference helpers (column-major, n x n / m x n) */
static double rnd_fill(double *x, size_t n, unsigned *s) {
  double m = 0;
  for (size_t i = 0; i < n; ++i) {
    *s = *s * 1103515245u + 12345u;
    x[i] = ((*s >> 8) & 0xffff) / 65536.0 - 0.5;
    m = fmax(m, fabs(x[i]));
  }
  return m;
}

/* dtrmm: B := alpha op(A) B / alpha B op(A), A triangular (ragged 300 with nb 128) */
static void test_dtrmm(dplasma_context_t *ctx, int side, int uplo, int trans, int diag) {
  const int nb = 128, M = 300, N = 250, ka = side == dplasmaLeft ? M : N;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, ka, ka), *B = dmat(ctx, dplasmaRealDouble, nb, M, N);
  double *a = malloc(sizeof(double) * ka * ka), *b = malloc(sizeof(double) * M * N), *r = malloc(sizeof(double) * M * N);
  unsigned sd = 7 + side + uplo + trans + diag;
  rnd_fill(a, (size_t)ka * ka, &sd);
  rnd_fill(b, (size_t)M * N, &sd);
  dplasma_desc_set_lapack(A, a, ka);
  dplasma_desc_set_lapack(B, b, M);
  const double alpha = 0.75;
  CHECK(dplasma_dtrmm(ctx, side, uplo, trans, diag, alpha, A, B) == 0, "dtrmm: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, r, M);
  double err = 0;
#define TA(i, j) (((uplo == dplasmaLower) ? (i) >= (j) : (i) <= (j)) ? ((i) == (j) && diag == dplasmaUnit ? 1.0 : a[(i) + (size_t)(j) * ka]) : 0.0)
#define OPA(i, j) (trans == dplasmaNoTrans ? TA(i, j) : TA(j, i))
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      if (side == dplasmaLeft)
        for (int k = 0; k < M; ++k) s += OPA(i, k) * b[k + (size_t)j * M];
      else
        for (int k = 0; k < N; ++k) s += b[i + (size_t)k * M] * OPA(k, j);
      err = fmax(err, fabs(alpha * s - r[i + (size_t)j * M]));
    }
#undef OPA
#undef TA
  printf("dtrmm %c%c%c%c max error %.3e\n", side == dplasmaLeft ? 'L' : 'R', uplo == dplasmaLower ? 'L' : 'U',
         trans == dplasmaNoTrans ? 'N' : 'T', diag == dplasmaUnit ? 'U' : 'N', err);
  CHECK(err < 1e-12, "dtrmm error %.3e", err);
  free(a), free(b), free(r);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

/* dsymm (left, lower) and zhemm (right, upper): the unused triangle of A holds garbage that must be ignored */
static void test_symm_hemm(dplasma_context_t *ctx) {
  const int nb = 128, M = 260, N = 190;
  {
    dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, M, M), *B = dmat(ctx, dplasmaRealDouble, nb, M, N);
    dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, M, N);
    double *a = malloc(sizeof(double) * M * M), *b = malloc(sizeof(double) * M * N), *c = malloc(sizeof(double) * M * N);
    double *r = malloc(sizeof(double) * M * N);
    unsigned sd = 99;
    rnd_fill(a, (size_t)M * M, &sd), rnd_fill(b, (size_t)M * N, &sd), rnd_fill(c, (size_t)M * N, &sd);
    dplasma_desc_set_lapack(A, a, M), dplasma_desc_set_lapack(B, b, M), dplasma_desc_set_lapack(C, c, M);
    CHECK(dplasma_dsymm(ctx, dplasmaLeft, dplasmaLower, 1.25, A, B, -0.5, C) == 0, "dsymm: %s", dplasma_last_error());
    dplasma_desc_get_lapack(C, r, M);
    double err = 0;
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < M; ++i) {
        double s = 0;
        for (int k = 0; k < M; ++k) s += (i >= k ? a[i + (size_t)k * M] : a[k + (size_t)i * M]) * b[k + (size_t)j * M];
        err = fmax(err, fabs(1.25 * s - 0.5 * c[i + (size_t)j * M] - r[i + (size_t)j * M]));
      }
    printf("dsymm LL max error %.3e\n", err);
    CHECK(err < 1e-12, "dsymm error %.3e", err);
    free(a), free(b), free(c), free(r);
    dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(C);
  }
  {
    dplasma_desc_t *A = dmat(ctx, dplasmaComplexDouble, nb, N, N), *B = dmat(ctx, dplasmaComplexDouble, nb, M, N);
    dplasma_desc_t *C = dmat(ctx, dplasmaComplexDouble, nb, M, N);
    double complex *a = malloc(sizeof(double complex) * N * N), *b = malloc(sizeof(double complex) * M * N);
    double complex *c = malloc(sizeof(double complex) * M * N), *r = malloc(sizeof(double complex) * M * N);
    unsigned sd = 5;
    rnd_fill((double *)a, 2 * (size_t)N * N, &sd), rnd_fill((double *)b, 2 * (size_t)M * N, &sd);
    rnd_fill((double *)c, 2 * (size_t)M * N, &sd);
    dplasma_desc_set_lapack(A, a, N), dplasma_desc_set_lapack(B, b, M), dplasma_desc_set_lapack(C, c, M);
    const double complex al = 0.5 - 0.25 * I, be = 1.5;
    CHECK(dplasma_zhemm(ctx, dplasmaRight, dplasmaUpper, al, A, B, be, C) == 0, "zhemm: %s", dplasma_last_error());
    dplasma_desc_get_lapack(C, r, M);
    double err = 0;
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < M; ++i) {
        double complex s = 0;
        for (int k = 0; k < N; ++k) {
          const double complex h = k < j ? a[k + (size_t)j * N] : k > j ? conj(a[j + (size_t)k * N]) : creal(a[j + (size_t)j * N]);
          s += b[i + (size_t)k * M] * h;
        }
        err = fmax(err, cabs(al * s + be * c[i + (size_t)j * M] - r[i + (size_t)j * M]));
      }
    printf("zhemm RU max error %.3e\n", err);
    CHECK(err < 1e-12, "zhemm error %.3e", err);
    /* lanhe (frobenius) of the same A against the expanded host matrix */
    double f = 0;
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < N; ++i) {
        const double complex h = i < j ? a[i + (size_t)j * N] : i > j ? conj(a[j + (size_t)i * N]) : creal(a[i + (size_t)i * N]);
        f += creal(h * conj(h));
      }
    const double fn = dplasma_zlanhe(ctx, dplasmaFrobeniusNorm, dplasmaUpper, A);
    printf("zlanhe F %.12e host %.12e\n", fn, sqrt(f));
    CHECK(fabs(fn - sqrt(f)) < 1e-12 * sqrt(f), "zlanhe %.12e vs %.12e", fn, sqrt(f));
    free(a), free(b), free(c), free(r);
    dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(C);
  }
}

/* dgetrf_1d + dgetrs (both transposes) and dgesv_1d on a ragged matrix; the pivots must be 1-based,
 * in range, and P A = L U must hold */
static void test_dgetrf(dplasma_context_t *ctx) {
  const int n = 700, nb = 256, nrhs = 5;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, 1, nb, 1, n, 1, 1);
  CHECK(IP != NULL, "desc_ipiv: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * n * n), *lu = malloc(sizeof(double) * n * n);
  double *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  int *ipiv = malloc(sizeof(int) * n);
  unsigned sd = 31;
  rnd_fill(a, (size_t)n * n, &sd), rnd_fill(b, (size_t)n * nrhs, &sd);
  for (int t = 0; t < 3; ++t) {
    const int trans = t == 1 ? dplasmaTrans : dplasmaNoTrans;
    dplasma_desc_set_lapack(A, a, n);
    dplasma_desc_set_lapack(B, b, n);
    int info;
    if (t < 2) {
      info = dplasma_dgetrf_1d(ctx, A, IP);
      CHECK(info == 0, "dgetrf_1d info %d (%s)", info, dplasma_last_error());
      CHECK(dplasma_dgetrs(ctx, trans, A, IP, B) == 0, "dgetrs: %s", dplasma_last_error());
    } else {
      info = dplasma_dgesv_1d(ctx, A, IP, B);
      CHECK(info == 0, "dgesv_1d info %d (%s)", info, dplasma_last_error());
    }
    dplasma_desc_get_lapack(B, x, n);
    dplasma_desc_get_lapack(IP, ipiv, 1);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += ipiv[i] < i + 1 || ipiv[i] > n;
    CHECK(bad == 0, "ipiv out of range (%d)", bad);
    double err = 0, bn = 0;
    for (int c = 0; c < nrhs; ++c)
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += (trans == dplasmaNoTrans ? a[i + (size_t)k * n] : a[k + (size_t)i * n]) * x[k + (size_t)c * n];
        err = fmax(err, fabs(s - b[i + (size_t)c * n]));
        bn = fmax(bn, fabs(b[i + (size_t)c * n]));
      }
    printf("%s n=%d nb=%d ||op(A)x-b||/||b|| %.3e\n", t == 2 ? "dgesv_1d" : trans == dplasmaNoTrans ? "dgetrs N" : "dgetrs T",
           n, nb, err / bn);
    CHECK(err / bn < 1e-9, "getrf/getrs residual %.3e", err / bn);
  }
  /* a corrupt pivot (past the last row) is reported by the row-move kernels (info -1001), never dereferenced:
   * dgetrs fails and names it */
  ipiv[300] = n + 40;
  dplasma_desc_set_lapack(IP, ipiv, 1);
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dgetrs(ctx, dplasmaNoTrans, A, IP, B) != 0, "dgetrs accepted a pivot past the last row");
  CHECK(strstr(dplasma_last_error(), "-1001") != NULL, "dgetrs corrupt pivot: unexpected error '%s'",
        dplasma_last_error());
  printf("dgetrs corrupt pivot -> %s\n", dplasma_last_error());
  free(a), free(lu), free(b), free(x), free(ipiv);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(IP);
}

/* dgetrf_nopiv on a diagonally dominant ragged matrix: L U = A (L unit lower, U upper, in place) */
static void test_dgetrf_nopiv(dplasma_context_t *ctx) {
  const int n = 600, nb = 128;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  double *a = malloc(sizeof(double) * n * n), *lu = malloc(sizeof(double) * n * n);
  unsigned sd = 5;
  rnd_fill(a, (size_t)n * n, &sd);
  for (int i = 0; i < n; ++i) a[i + (size_t)i * n] += n;
  dplasma_desc_set_lapack(A, a, n);
  const int info = dplasma_dgetrf_nopiv(ctx, A);
  CHECK(info == 0, "dgetrf_nopiv info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, lu, n);
  double err = 0, an = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      const int kk = i < j ? i : j;
      for (int k = 0; k <= kk; ++k) s += (k == i ? 1.0 : lu[i + (size_t)k * n]) * lu[k + (size_t)j * n];
      err = fmax(err, fabs(s - a[i + (size_t)j * n]));
      an = fmax(an, fabs(a[i + (size_t)j * n]));
    }
  printf("dgetrf_nopiv n=%d nb=%d: ||LU - A|| / ||A|| %.3e\n", n, nb, err / an);
  CHECK(err / an < 1e-13, "getrf_nopiv residual %.3e", err / an);
  free(a), free(lu);
  dplasma_desc_destroy(A);
}

/* flat-tree LQ family on a wide matrix: gelqf, unglq (Q Q^T = I, L Q = A), unmlq (left Q x, right A Q^T = [L 0]),
 * minimum-norm gels / gelqs (A x = b) */
static void test_dgelqf(dplasma_context_t *ctx) {
  const int m = 400, n = 700, nb = 128, ib = 32, nrhs = 3;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *T = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1,
                                               dplasmaUpperLower);
  dplasma_desc_t *Q = dmat(ctx, dplasmaRealDouble, nb, m, n), *C = dmat(ctx, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *X = dmat(ctx, dplasmaRealDouble, nb, n, nrhs), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  CHECK(T && Q && C && X && B, "descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * m * n), *f = malloc(sizeof(double) * m * n), *q = malloc(sizeof(double) * m * n);
  double *c = malloc(sizeof(double) * m * n), *x = malloc(sizeof(double) * n * nrhs), *y = malloc(sizeof(double) * n * nrhs);
  double *b = malloc(sizeof(double) * n * nrhs);
  unsigned sd = 91;
  rnd_fill(a, (size_t)m * n, &sd), rnd_fill(x, (size_t)n * nrhs, &sd), rnd_fill(b, (size_t)n * nrhs, &sd);
  dplasma_desc_set_lapack(A, a, m);
  int info = dplasma_dgelqf(ctx, A, T);
  CHECK(info == 0, "dgelqf info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, f, m);
  CHECK(dplasma_dunglq(ctx, A, T, Q) == 0, "dunglq: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Q, q, m);
  double orth = 0, res = 0, an = 0;
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += q[i + (size_t)k * m] * q[j + (size_t)k * m];
      orth = fmax(orth, fabs(s - (i == j)));
    }
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k <= i; ++k) s += f[i + (size_t)k * m] * q[k + (size_t)j * m];
      res = fmax(res, fabs(s - a[i + (size_t)j * m]));
      an = fmax(an, fabs(a[i + (size_t)j * m]));
    }
  printf("dgelqf m=%d n=%d nb=%d ib=%d: ||Q Q^T - I|| %.3e  ||LQ - A||/||A|| %.3e\n", m, n, nb, ib, orth, res / an);
  CHECK(orth < 1e-12 && res / an < 1e-12, "gelqf / unglq residuals");
  /* A0 Q^T = [L 0] (right, transposed) */
  dplasma_desc_set_lapack(C, a, m);
  CHECK(dplasma_dunmlq(ctx, dplasmaRight, dplasmaTrans, A, T, C) == 0, "dunmlq R T: %s", dplasma_last_error());
  dplasma_desc_get_lapack(C, c, m);
  double e1 = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) e1 = fmax(e1, fabs(c[i + (size_t)j * m] - (j <= i ? f[i + (size_t)j * m] : 0.0)));
  /* Q^T x (left, transposed): the first m entries are (Q x-rows) = q x */
  dplasma_desc_set_lapack(X, x, n);
  CHECK(dplasma_dunmlq(ctx, dplasmaLeft, dplasmaNoTrans, A, T, X) == 0, "dunmlq L N: %s", dplasma_last_error());
  dplasma_desc_get_lapack(X, y, n);
  double e2 = 0;
  for (int r = 0; r < nrhs; ++r)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += q[i + (size_t)k * m] * x[k + (size_t)r * n];
      e2 = fmax(e2, fabs(s - y[i + (size_t)r * n]));
    }
  printf("dunmlq: ||A Q^T - [L 0]|| / ||A|| %.3e   ||(Q x)(0:m) - Q1 x|| %.3e\n", e1 / an, e2);
  CHECK(e1 / an < 1e-12 && e2 < 1e-11, "unmlq residuals");
  /* minimum norm: A x = b(0:m) */
  dplasma_desc_set_lapack(A, a, m);
  dplasma_desc_set_lapack(B, b, n);
  info = dplasma_dgels(ctx, dplasmaNoTrans, A, T, B);
  CHECK(info == 0, "dgels (M < N) info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(B, y, n);
  double ge = 0;
  for (int r = 0; r < nrhs; ++r)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * m] * y[k + (size_t)r * n];
      ge = fmax(ge, fabs(s - b[i + (size_t)r * n]));
    }
  /* gelqs on the factored A (from the gels call) with fresh b: same solution */
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dgelqs(ctx, A, T, B) == 0, "dgelqs: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, c, n);
  double de = 0;
  for (int r = 0; r < nrhs; ++r)
    for (int i = 0; i < n; ++i) de = fmax(de, fabs(c[i + (size_t)r * n] - y[i + (size_t)r * n]));
  printf("dgels min-norm m=%d n=%d: ||A x - b|| %.3e  gelqs vs gels %.3e\n", m, n, ge, de);
  CHECK(ge < 1e-10 && de < 1e-12, "gels / gelqs residuals");
  free(a), free(f), free(q), free(c), free(x), free(y), free(b);
  dplasma_desc_destroy(A), dplasma_desc_destroy(T), dplasma_desc_destroy(Q), dplasma_desc_destroy(C);
  dplasma_desc_destroy(X), dplasma_desc_destroy(B);
}

/* complex LQ: the conjugate-transpose construction must give L Q = A with Q Q^H = I */
static void test_zgelqf(dplasma_context_t *ctx) {
  const int m = 200, n = 330, nb = 64, ib = 16;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaComplexDouble, nb, m, n), *Q = dmat(ctx, dplasmaComplexDouble, nb, m, n);
  dplasma_desc_t *T = dplasma_desc_block_cyclic(ctx, dplasmaComplexDouble, ib, nb, mt * ib, nt * nb, 1, 1,
                                               dplasmaUpperLower);
  CHECK(A && Q && T, "descriptors: %s", dplasma_last_error());
  double complex *a = malloc(sizeof(double complex) * m * n), *f = malloc(sizeof(double complex) * m * n);
  double complex *q = malloc(sizeof(double complex) * m * n);
  double *re = malloc(sizeof(double) * 2 * m * n);
  unsigned sd = 17;
  rnd_fill(re, (size_t)2 * m * n, &sd);
  for (size_t i = 0; i < (size_t)m * n; ++i) a[i] = re[2 * i] + I * re[2 * i + 1];
  dplasma_desc_set_lapack(A, a, m);
  CHECK(dplasma_zgelqf(ctx, A, T) == 0, "zgelqf: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, f, m);
  CHECK(dplasma_zunglq(ctx, A, T, Q) == 0, "zunglq: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Q, q, m);
  double orth = 0, res = 0, an = 0;
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < m; ++i) {
      double complex s = 0;
      for (int k = 0; k < n; ++k) s += q[i + (size_t)k * m] * conj(q[j + (size_t)k * m]);
      orth = fmax(orth, cabs(s - (i == j)));
    }
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double complex s = 0;
      for (int k = 0; k <= i; ++k) s += f[i + (size_t)k * m] * q[k + (size_t)j * m];
      res = fmax(res, cabs(s - a[i + (size_t)j * m]));
      an = fmax(an, cabs(a[i + (size_t)j * m]));
    }
  printf("zgelqf m=%d n=%d: ||Q Q^H - I|| %.3e  ||LQ - A||/||A|| %.3e\n", m, n, orth, res / an);
  CHECK(orth < 1e-12 && res / an < 1e-12, "zgelqf / zunglq residuals");
  free(a), free(f), free(q), free(re);
  dplasma_desc_destroy(A), dplasma_desc_destroy(Q), dplasma_desc_destroy(T);
}

/* incremental-pivoting LU (tile GETRF / GESSM / TSTRF / SSSSM) + gesv_incpiv on a ragged matrix: A x = b */
static void test_dgesv_incpiv(dplasma_context_t *ctx) {
  const int n = 500, nb = 128, ib = 32, nrhs = 4;
  const int mt = (n + nb - 1) / nb, nt = mt;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_desc_t *L = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, n, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, nb, 1, n, nt, 1, 1);
  CHECK(A && B && L && IP, "incpiv descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  unsigned sd = 404;
  rnd_fill(a, (size_t)n * n, &sd), rnd_fill(b, (size_t)n * nrhs, &sd);
  dplasma_desc_set_lapack(A, a, n);
  dplasma_desc_set_lapack(B, b, n);
  const int info = dplasma_dgesv_incpiv(ctx, A, L, IP, B);
  CHECK(info == 0, "dgesv_incpiv info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(B, x, n);
  double err = 0, bn = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)c * n];
      err = fmax(err, fabs(s - b[i + (size_t)c * n]));
      bn = fmax(bn, fabs(b[i + (size_t)c * n]));
    }
  printf("dgesv_incpiv n=%d nb=%d ib=%d: ||Ax-b||/||b|| %.3e\n", n, nb, ib, err / bn);
  CHECK(err / bn < 1e-9, "gesv_incpiv residual %.3e", err / bn);
  /* the same solve in two halves: trsmpl_incpiv (L^-1 P b) and the upper TRSM */
  double *x2 = malloc(sizeof(double) * n * nrhs);
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dtrsmpl_incpiv(ctx, A, L, IP, B) == 0, "dtrsmpl_incpiv: %s", dplasma_last_error());
  CHECK(dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B) == 0, "trsm: %s",
        dplasma_last_error());
  dplasma_desc_get_lapack(B, x2, n);
  double d2 = 0, xn = 0;
  for (size_t e = 0; e < (size_t)n * nrhs; ++e) d2 = fmax(d2, fabs(x2[e] - x[e])), xn = fmax(xn, fabs(x[e]));
  printf("dtrsmpl_incpiv + dtrsm vs gesv_incpiv: max diff %.3e (|x| %.3e)\n", d2, xn);
  CHECK(d2 <= 1e-12 * xn, "dtrsmpl_incpiv differs (%.3e)", d2);
  free(a), free(b), free(x), free(x2);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(L), dplasma_desc_destroy(IP);
}

/* flat-tree QR family: geqrf, ungqr (thin and full Q), unmqr (left Q^T, right Q), gels */
static void test_dgeqrf(dplasma_context_t *ctx) {
  const int m = 700, n = 400, nb = 128, ib = 32, nrhs = 3, p = 50;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *T = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1,
                                               dplasmaUpperLower);
  dplasma_desc_t *Q = dmat(ctx, dplasmaRealDouble, nb, m, n), *Qf = dmat(ctx, dplasmaRealDouble, nb, m, m);
  dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, m, n), *D = dmat(ctx, dplasmaRealDouble, nb, p, m);
  dplasma_desc_t *B = dmat(ctx, dplasmaRealDouble, nb, m, nrhs);
  CHECK(T && Q && Qf && C && D && B, "descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * m * n), *f = malloc(sizeof(double) * m * n), *q = malloc(sizeof(double) * m * n);
  double *qf = malloc(sizeof(double) * m * m), *c = malloc(sizeof(double) * m * n);
  double *d = malloc(sizeof(double) * p * m), *dq = malloc(sizeof(double) * p * m);
  double *b = malloc(sizeof(double) * m * nrhs), *x = malloc(sizeof(double) * m * nrhs);
  unsigned sd = 77;
  rnd_fill(a, (size_t)m * n, &sd), rnd_fill(d, (size_t)p * m, &sd), rnd_fill(b, (size_t)m * nrhs, &sd);
  dplasma_desc_set_lapack(A, a, m);
  int info = dplasma_dgeqrf(ctx, A, T);
  CHECK(info == 0, "dgeqrf info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, f, m);
  CHECK(dplasma_dungqr(ctx, A, T, Q) == 0, "dungqr: %s", dplasma_last_error());
  CHECK(dplasma_dungqr(ctx, A, T, Qf) == 0, "dungqr full: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Q, q, m);
  dplasma_desc_get_lapack(Qf, qf, m);
  double orth = 0, res = 0, an = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += q[k + (size_t)i * m] * q[k + (size_t)j * m];
      orth = fmax(orth, fabs(s - (i == j)));
    }
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k <= j && k < n; ++k) s += q[i + (size_t)k * m] * f[k + (size_t)j * m];
      res = fmax(res, fabs(s - a[i + (size_t)j * m]));
      an = fmax(an, fabs(a[i + (size_t)j * m]));
    }
  printf("dgeqrf m=%d n=%d nb=%d ib=%d: ||Q^T Q - I|| %.3e  ||QR - A||/||A|| %.3e\n", m, n, nb, ib, orth, res / an);
  CHECK(orth < 1e-12 && res / an < 1e-12, "geqrf / ungqr residuals");
  /* Q^T A0 = [R; 0] */
  dplasma_desc_set_lapack(C, a, m);
  CHECK(dplasma_dunmqr(ctx, dplasmaLeft, dplasmaTrans, A, T, C) == 0, "dunmqr L T: %s", dplasma_last_error());
  dplasma_desc_get_lapack(C, c, m);
  double e1 = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) e1 = fmax(e1, fabs(c[i + (size_t)j * m] - (i <= j ? f[i + (size_t)j * m] : 0.0)));
  /* D Q (right, no transpose) against the host product with the full Q */
  dplasma_desc_set_lapack(D, d, p);
  CHECK(dplasma_dunmqr(ctx, dplasmaRight, dplasmaNoTrans, A, T, D) == 0, "dunmqr R N: %s", dplasma_last_error());
  dplasma_desc_get_lapack(D, dq, p);
  double e2 = 0;
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < p; ++i) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += d[i + (size_t)k * p] * qf[k + (size_t)j * m];
      e2 = fmax(e2, fabs(s - dq[i + (size_t)j * p]));
    }
  printf("dunmqr: ||Q^T A - R|| / ||A|| %.3e   ||D Q - D*Q|| %.3e\n", e1 / an, e2);
  CHECK(e1 / an < 1e-12 && e2 < 1e-11, "unmqr residuals");
  /* least squares: A^T (A x - b) = 0 */
  dplasma_desc_set_lapack(A, a, m);
  dplasma_desc_set_lapack(B, b, m);
  info = dplasma_dgels(ctx, dplasmaNoTrans, A, T, B);
  CHECK(info == 0, "dgels info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(B, x, m);
  double ne = 0, bn = 0;
  for (int r = 0; r < nrhs; ++r) {
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int i = 0; i < m; ++i) {
        double ax = 0;
        for (int k = 0; k < n; ++k) ax += a[i + (size_t)k * m] * x[k + (size_t)r * m];
        s += a[i + (size_t)j * m] * (ax - b[i + (size_t)r * m]);
      }
      ne = fmax(ne, fabs(s));
    }
    for (int i = 0; i < m; ++i) bn = fmax(bn, fabs(b[i + (size_t)r * m]));
  }
  printf("dgels: ||A^T (A x - b)|| / (m ||A|| ||b||) %.3e\n", ne / (m * an * bn));
  CHECK(ne / (m * an * bn) < 1e-12, "gels normal equations %.3e", ne / (m * an * bn));
  free(a), free(f), free(q), free(qf), free(c), free(d), free(dq), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(T), dplasma_desc_destroy(Q), dplasma_desc_destroy(Qf);
  dplasma_desc_destroy(C), dplasma_desc_destroy(D), dplasma_desc_destroy(B);
}


/* tree-driven QR / LQ (native_qrtree.cpp trees + native.cpp *_param builders) on ragged matrices.  Trees: HQR with
 * a greedy low tree over TS domains of a = 2 tiles and a flat high tree over p = 3 virtual process rows (TS, local
 * TT and distributed TT kills), HQR binary/greedy with domino, systolic, adaptive SVD.  Checks: ||Q^T Q - I||,
 * ||QR - A|| (ungqr_param), |R| equal to the flat geqrf's |R| (R is unique up to row signs), Q^T A0 = [R; 0] and
 * D Q against the host product (unmqr_param), the least-squares normal equations (geqrs_param). */
static void test_dgeqrf_param(dplasma_context_t *ctx) {
  const int m = 900, n = 500, nb = 128, ib = 32, nrhs = 2, p = 40;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, m, n), *F = dmat(ctx, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *TS = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *TT = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *T0 = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *Q = dmat(ctx, dplasmaRealDouble, nb, m, n), *Qf = dmat(ctx, dplasmaRealDouble, nb, m, m);
  dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, m, n), *D = dmat(ctx, dplasmaRealDouble, nb, p, m);
  dplasma_desc_t *B = dmat(ctx, dplasmaRealDouble, nb, m, nrhs);
  CHECK(A && F && TS && TT && T0 && Q && Qf && C && D && B, "param descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * m * n), *f = malloc(sizeof(double) * m * n), *f0 = malloc(sizeof(double) * m * n);
  double *q = malloc(sizeof(double) * m * n), *qf = malloc(sizeof(double) * m * m), *c = malloc(sizeof(double) * m * n);
  double *d = malloc(sizeof(double) * p * m), *dq = malloc(sizeof(double) * p * m);
  double *b = malloc(sizeof(double) * m * nrhs), *x = malloc(sizeof(double) * m * nrhs);
  unsigned sd = 313;
  rnd_fill(a, (size_t)m * n, &sd), rnd_fill(d, (size_t)p * m, &sd), rnd_fill(b, (size_t)m * nrhs, &sd);
  dplasma_desc_set_lapack(F, a, m);
  CHECK(dplasma_dgeqrf(ctx, F, T0) == 0, "flat dgeqrf: %s", dplasma_last_error());
  dplasma_desc_get_lapack(F, f0, m);
  double an = 0;
  for (size_t e = 0; e < (size_t)m * n; ++e) an = fmax(an, fabs(a[e]));
  for (int kind = 0; kind < 5; ++kind) {
    dplasma_qrtree_t qt;
    memset(&qt, 0, sizeof qt);
    int rc;
    const char *nm;
    if (kind == 0) rc = dplasma_hqr_init(&qt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 2, 3, 0, 0), nm = "hqr greedy/flat a=2 p=3";
    else if (kind == 1) rc = dplasma_hqr_init(&qt, dplasmaNoTrans, A, 3, DPLASMA_GREEDY_TREE, 1, 2, 1, 0), nm = "hqr binary/greedy p=2 domino";
    else if (kind == 2) rc = dplasma_systolic_init(&qt, dplasmaNoTrans, A, 2, 2), nm = "systolic 2x2";
    else if (kind == 3) rc = dplasma_svd_init(&qt, dplasmaNoTrans, A, 2, 2, 2, 1), nm = "svd fibonacci p=2";
    else rc = dplasma_hqr_init(&qt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 4, 1, 0, 0), nm = "hqr greedy a=4";
    CHECK(rc == 0, "%s init: %s", nm, dplasma_last_error());
    if (rc) continue;
    CHECK(qt.mt == mt && qt.nt == nt, "%s dims %d x %d", nm, qt.mt, qt.nt);
    CHECK(dplasma_qrtree_check(A, &qt) == 0, "%s check: %s", nm, dplasma_last_error());
    dplasma_desc_set_lapack(A, a, m);
    int info = dplasma_dgeqrf_param(ctx, &qt, A, TS, TT);
    CHECK(info == 0, "%s dgeqrf_param info %d (%s)", nm, info, dplasma_last_error());
    dplasma_desc_get_lapack(A, f, m);
    CHECK(dplasma_dungqr_param(ctx, &qt, A, TS, TT, Q) == 0, "%s dungqr_param: %s", nm, dplasma_last_error());
    CHECK(dplasma_dungqr_param(ctx, &qt, A, TS, TT, Qf) == 0, "%s dungqr_param full: %s", nm, dplasma_last_error());
    dplasma_desc_get_lapack(Q, q, m);
    dplasma_desc_get_lapack(Qf, qf, m);
    double orth = 0, res = 0, rd = 0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < m; ++k) s += q[k + (size_t)i * m] * q[k + (size_t)j * m];
        orth = fmax(orth, fabs(s - (i == j)));
      }
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < m; ++i) {
        double s = 0;
        for (int k = 0; k <= j && k < n; ++k) s += q[i + (size_t)k * m] * f[k + (size_t)j * m];
        res = fmax(res, fabs(s - a[i + (size_t)j * m]));
        if (i <= j) rd = fmax(rd, fabs(fabs(f[i + (size_t)j * m]) - fabs(f0[i + (size_t)j * m])));
      }
    /* Q^T A0 = [R; 0] and D Q against the host product with the full Q */
    dplasma_desc_set_lapack(C, a, m);
    CHECK(dplasma_dunmqr_param(ctx, dplasmaLeft, dplasmaTrans, &qt, A, TS, TT, C) == 0, "%s dunmqr_param L T: %s", nm,
          dplasma_last_error());
    dplasma_desc_get_lapack(C, c, m);
    double e1 = 0, e2 = 0;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < m; ++i) e1 = fmax(e1, fabs(c[i + (size_t)j * m] - (i <= j ? f[i + (size_t)j * m] : 0.0)));
    dplasma_desc_set_lapack(D, d, p);
    CHECK(dplasma_dunmqr_param(ctx, dplasmaRight, dplasmaNoTrans, &qt, A, TS, TT, D) == 0, "%s dunmqr_param R N: %s", nm,
          dplasma_last_error());
    dplasma_desc_get_lapack(D, dq, p);
    for (int j = 0; j < m; ++j)
      for (int i = 0; i < p; ++i) {
        double s = 0;
        for (int k = 0; k < m; ++k) s += d[i + (size_t)k * p] * qf[k + (size_t)j * m];
        e2 = fmax(e2, fabs(s - dq[i + (size_t)j * p]));
      }
    /* least squares on the factored A: A^T (A x - b) = 0 */
    dplasma_desc_set_lapack(B, b, m);
    CHECK(dplasma_dgeqrs_param(ctx, &qt, A, TS, TT, B) == 0, "%s dgeqrs_param: %s", nm, dplasma_last_error());
    dplasma_desc_get_lapack(B, x, m);
    double ne = 0, bn = 0;
    for (int r = 0; r < nrhs; ++r) {
      for (int j = 0; j < n; ++j) {
        double s = 0;
        for (int i = 0; i < m; ++i) {
          double ax = 0;
          for (int k = 0; k < n; ++k) ax += a[i + (size_t)k * m] * x[k + (size_t)r * m];
          s += a[i + (size_t)j * m] * (ax - b[i + (size_t)r * m]);
        }
        ne = fmax(ne, fabs(s));
      }
      for (int i = 0; i < m; ++i) bn = fmax(bn, fabs(b[i + (size_t)r * m]));
    }
    printf("dgeqrf_param %-30s ||Q^T Q - I|| %.2e ||QR - A||/||A|| %.2e | |R| - |R_flat| | %.2e  Q^T A %.2e  D Q %.2e  "
           "geqrs %.2e\n", nm, orth, res / an, rd / an, e1 / an, e2, ne / (m * an * bn));
    CHECK(orth < 1e-12 && res / an < 1e-12 && rd / an < 1e-11 && e1 / an < 1e-12 && e2 < 1e-11 &&
          ne / (m * an * bn) < 1e-12, "%s residuals", nm);
    dplasma_hqr_finalize(&qt);   /* (every init's finalize releases the native tree) */
  }
  free(a), free(f), free(f0), free(q), free(qf), free(c), free(d), free(dq), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(F), dplasma_desc_destroy(TS), dplasma_desc_destroy(TT);
  dplasma_desc_destroy(T0), dplasma_desc_destroy(Q), dplasma_desc_destroy(Qf), dplasma_desc_destroy(C);
  dplasma_desc_destroy(D), dplasma_desc_destroy(B);
}

/* tree-driven LQ on a wide ragged matrix (tree built with trans = Trans: over A's tile columns): gelqf_param,
 * unglq_param (Q Q^T = I, LQ = A), unmlq_param (A0 Q^T = [L 0]), gelqs_param (minimum-norm A x = b) */
static void test_dgelqf_param(dplasma_context_t *ctx) {
  const int m = 300, n = 800, nb = 128, ib = 32, nrhs = 2;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, m, n), *Q = dmat(ctx, dplasmaRealDouble, nb, m, n);
  dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, m, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_desc_t *TS = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *TT = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  CHECK(A && Q && C && B && TS && TT, "lq param descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * m * n), *f = malloc(sizeof(double) * m * n), *q = malloc(sizeof(double) * m * n);
  double *c = malloc(sizeof(double) * m * n), *b = malloc(sizeof(double) * n * nrhs), *y = malloc(sizeof(double) * n * nrhs);
  unsigned sd = 515;
  rnd_fill(a, (size_t)m * n, &sd), rnd_fill(b, (size_t)n * nrhs, &sd);
  dplasma_qrtree_t qt;
  memset(&qt, 0, sizeof qt);
  CHECK(dplasma_hqr_init(&qt, dplasmaTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 2, 2, 0, 1) == 0, "lq tree: %s",
        dplasma_last_error());
  CHECK(qt.mt == nt && qt.nt == mt, "lq tree dims %d x %d", qt.mt, qt.nt);
  dplasma_desc_set_lapack(A, a, m);
  int info = dplasma_dgelqf_param(ctx, &qt, A, TS, TT);
  CHECK(info == 0, "dgelqf_param info %d (%s)", info, dplasma_last_error());
  dplasma_desc_get_lapack(A, f, m);
  CHECK(dplasma_dunglq_param(ctx, &qt, A, TS, TT, Q) == 0, "dunglq_param: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Q, q, m);
  double orth = 0, res = 0, an = 0;
  for (int j = 0; j < m; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += q[i + (size_t)k * m] * q[j + (size_t)k * m];
      orth = fmax(orth, fabs(s - (i == j)));
    }
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k <= i; ++k) s += f[i + (size_t)k * m] * q[k + (size_t)j * m];
      res = fmax(res, fabs(s - a[i + (size_t)j * m]));
      an = fmax(an, fabs(a[i + (size_t)j * m]));
    }
  dplasma_desc_set_lapack(C, a, m);
  CHECK(dplasma_dunmlq_param(ctx, dplasmaRight, dplasmaTrans, &qt, A, TS, TT, C) == 0, "dunmlq_param R T: %s",
        dplasma_last_error());
  dplasma_desc_get_lapack(C, c, m);
  double e1 = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) e1 = fmax(e1, fabs(c[i + (size_t)j * m] - (j <= i ? f[i + (size_t)j * m] : 0.0)));
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dgelqs_param(ctx, &qt, A, TS, TT, B) == 0, "dgelqs_param: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, y, n);
  double ge = 0;
  for (int r = 0; r < nrhs; ++r)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * m] * y[k + (size_t)r * n];
      ge = fmax(ge, fabs(s - b[i + (size_t)r * n]));
    }
  printf("dgelqf_param hqr greedy/flat tsrr: ||Q Q^T - I|| %.2e ||LQ - A||/||A|| %.2e  A Q^T %.2e  gelqs ||Ax-b|| %.2e\n",
         orth, res / an, e1 / an, ge);
  CHECK(orth < 1e-12 && res / an < 1e-12 && e1 / an < 1e-12 && ge < 1e-10, "gelqf_param residuals");
  dplasma_hqr_finalize(&qt);
  free(a), free(f), free(q), free(c), free(b), free(y);
  dplasma_desc_destroy(A), dplasma_desc_destroy(Q), dplasma_desc_destroy(C), dplasma_desc_destroy(B);
  dplasma_desc_destroy(TS), dplasma_desc_destroy(TT);
}

/* hybrid LU-QR (native getrf_qrf + trsmpl_qrf, HQR greedy tree a = 4): per criterion the lu_tab pattern (DEFAULT
 * alternates, LU_ONLY / QR_ONLY, RANDOM balanced, HIGHAM / MUMPS on one process row: LU unless singular) and the
 * solve x = U^-1 trsmpl_qrf(b) checked as ||A x - b|| / (||A|| ||x|| n) (tests/testing_zgetrf_qrf.c) */
static void test_dgetrf_qrf(dplasma_context_t *ctx) {
  const int n = 900, nb = 128, ib = 32, nrhs = 3;
  const int mt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_desc_t *TS = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, mt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *TT = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, mt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, nb, 1, mt * nb, mt, 1, 1);
  CHECK(A && B && TS && TT && IP, "getrf_qrf descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  unsigned sd = 733;
  rnd_fill(a, (size_t)n * n, &sd), rnd_fill(b, (size_t)n * nrhs, &sd);
  dplasma_qrtree_t qt;
  memset(&qt, 0, sizeof qt);
  CHECK(dplasma_hqr_init(&qt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 4, 1, 0, 0) == 0, "tree: %s",
        dplasma_last_error());
  const int crit[] = {0, 3, 4, 5, 1, 2};
  const double alph[] = {1.0, 1.0, 1.0, 50.0, 1.0, 1.0};
  const char *names[] = {"DEFAULT", "LU_ONLY", "QR_ONLY", "RANDOM 50%", "HIGHAM", "MUMPS"};
  for (int c = 0; c < 6; ++c) {
    int lu_tab[64], info = -7;
    memset(lu_tab, 0xff, sizeof lu_tab);
    dplasma_desc_set_lapack(A, a, n);
    int rc = dplasma_dgetrf_qrf(ctx, &qt, A, IP, TS, TT, crit[c], alph[c], lu_tab, &info);
    CHECK(rc == 0 && info == 0, "dgetrf_qrf %s rc %d info %d (%s)", names[c], rc, info, dplasma_last_error());
    int nlu = 0, pat = 1;
    char tab[80];
    for (int k = 0; k < mt; ++k) {
      nlu += lu_tab[k] == 1;
      tab[k] = lu_tab[k] == 1 ? 'L' : (lu_tab[k] == 0 ? 'Q' : '?');
      if (crit[c] == 0 && lu_tab[k] != k % 2) pat = 0;
      if ((crit[c] == 3 || crit[c] == 1 || crit[c] == 2) && lu_tab[k] != 1) pat = 0;
      if (crit[c] == 4 && lu_tab[k] != 0) pat = 0;
    }
    tab[mt] = 0;
    if (crit[c] == 5 && nlu != (int)lround(mt * 0.5)) pat = 0;
    dplasma_desc_set_lapack(B, b, n);
    CHECK(dplasma_dtrsmpl_qrf(ctx, &qt, A, IP, B, TS, TT, lu_tab) == 0, "dtrsmpl_qrf %s: %s", names[c], dplasma_last_error());
    CHECK(dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B) == 0, "trsm: %s",
          dplasma_last_error());
    dplasma_desc_get_lapack(B, x, n);
    double err = 0, an = 0, xn = 0;
    for (size_t e = 0; e < (size_t)n * n; ++e) an = fmax(an, fabs(a[e]));
    for (int r = 0; r < nrhs; ++r)
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)r * n];
        err = fmax(err, fabs(s - b[i + (size_t)r * n]));
        xn = fmax(xn, fabs(x[i + (size_t)r * n]));
      }
    const double rel = err / (an * xn * n);
    printf("dgetrf_qrf %-10s lu_tab %s  ||Ax-b||/(||A|| ||x|| n) %.2e\n", names[c], tab, rel);
    CHECK(pat && rel < 1e-15, "getrf_qrf %s: pattern %d residual %.3e", names[c], pat, rel);
  }
  dplasma_hqr_finalize(&qt);
  free(a), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(TS), dplasma_desc_destroy(TT);
  dplasma_desc_destroy(IP);
}

/* getrf_qrf with data-dependent criteria on a p = 2 domain period (DPLASMA_LUQR_P): the same matrix as
 * tests/test_lu_qr.py _luqr_run (plrnt seed 7, N 1536, NB 256, HQR greedy/flat a = 2 p = 2); prints lu_tab per
 * (criterion, alpha) and dumps the factors under DPLASMA_TEST_DUMP for tests/test_capi.py to compare with the Python
 * engine; solve residual checked here */
static void test_dgetrf_qrf_criteria(dplasma_context_t *ctx) {
  const int n = 1536, nb = 256, ib = 32, nrhs = 2;
  const int mt = n / nb;
  setenv("DPLASMA_LUQR_P", "2", 1);
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_desc_t *TS = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, n, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *TT = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, n, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, nb, 1, n, mt, 1, 1);
  CHECK(A && B && TS && TT && IP, "getrf_qrf criteria descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * n * n), *f = malloc(sizeof(double) * n * n);
  double *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  CHECK(dplasma_dplrnt(ctx, 0, A, 7) == 0 && dplasma_dplrnt(ctx, 0, B, 8) == 0, "plrnt: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  dplasma_desc_get_lapack(B, b, n);
  dplasma_qrtree_t qt;
  memset(&qt, 0, sizeof qt);
  CHECK(dplasma_hqr_init(&qt, dplasmaNoTrans, A, DPLASMA_GREEDY_TREE, DPLASMA_FLAT_TREE, 2, 2, 0, 0) == 0, "tree: %s",
        dplasma_last_error());
  const int crit[] = {1, 6, 7, 8, 2, 2};
  const double alph[] = {0.02, 1.0, 2.0, 4.0, 1.0, 3.0};
  const char *dump = getenv("DPLASMA_TEST_DUMP");
  for (int c = 0; c < 6; ++c) {
    int lu_tab[16], info = -7;
    dplasma_desc_set_lapack(A, a, n);
    int rc = dplasma_dgetrf_qrf(ctx, &qt, A, IP, TS, TT, crit[c], alph[c], lu_tab, &info);
    CHECK(rc == 0 && info == 0, "dgetrf_qrf crit %d rc %d info %d (%s)", crit[c], rc, info, dplasma_last_error());
    char tab[32];
    for (int k = 0; k < mt; ++k) tab[k] = lu_tab[k] ? 'L' : 'Q';
    tab[mt] = 0;
    dplasma_desc_get_lapack(A, f, n);
    if (dump) {
      char path[512];
      snprintf(path, sizeof path, "%s/luqr_%d_%g.bin", dump, crit[c], alph[c]);
      FILE *fp = fopen(path, "wb");
      if (fp) fwrite(f, sizeof(double), (size_t)n * n, fp), fclose(fp);
    }
    dplasma_desc_set_lapack(B, b, n);
    CHECK(dplasma_dtrsmpl_qrf(ctx, &qt, A, IP, B, TS, TT, lu_tab) == 0, "dtrsmpl_qrf: %s", dplasma_last_error());
    CHECK(dplasma_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B) == 0, "trsm: %s",
          dplasma_last_error());
    dplasma_desc_get_lapack(B, x, n);
    double err = 0, an = 0, xn = 0;
    for (size_t e = 0; e < (size_t)n * n; ++e) an = fmax(an, fabs(a[e]));
    for (int r = 0; r < nrhs; ++r)
      for (int i = 0; i < n; ++i) {
        double s = 0;
        for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)r * n];
        err = fmax(err, fabs(s - b[i + (size_t)r * n]));
        xn = fmax(xn, fabs(x[i + (size_t)r * n]));
      }
    printf("luqr_criteria crit=%d alpha=%g lu_tab=%s resid=%.2e\n", crit[c], alph[c], tab, err / (an * xn * n));
    CHECK(err / (an * xn * n) < 1e-15, "getrf_qrf crit %d residual", crit[c]);
  }
  unsetenv("DPLASMA_LUQR_P");
  dplasma_hqr_finalize(&qt);
  free(a), free(f), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B), dplasma_desc_destroy(TS), dplasma_desc_destroy(TT);
  dplasma_desc_destroy(IP);
}

/* eigenvalues natively: heev (herbt two-sided panel reduction to band + host bulge chase + QL) on the 1-D Laplacian
 * (known spectrum 2 - 2 cos(k pi / (n + 1))), on random symmetric / Hermitian matrices (trace and Frobenius invariants,
 * Lower and Upper agree), and hbrdt on a band descriptor (d, e similar to the band: the same invariants) */
static void test_heev(dplasma_context_t *ctx) {
  const int n = 600, nb = 64;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *W = dmat(ctx, dplasmaRealDouble, nb, n, 1);
  double *a = malloc(sizeof(double) * n * n), *w = malloc(sizeof(double) * n), *w2 = malloc(sizeof(double) * n);
  /* 1-D Laplacian */
  memset(a, 0, sizeof(double) * n * n);
  for (int i = 0; i < n; ++i) {
    a[i + (size_t)i * n] = 2.0;
    if (i + 1 < n) a[i + 1 + (size_t)i * n] = a[i + (size_t)(i + 1) * n] = -1.0;
  }
  dplasma_desc_set_lapack(A, a, n);
  CHECK(dplasma_dheev(ctx, dplasmaNoVec, dplasmaLower, A, W, NULL) == 0, "dheev: %s", dplasma_last_error());
  dplasma_desc_get_lapack(W, w, n);
  double el = 0;
  for (int k = 0; k < n; ++k) el = fmax(el, fabs(w[k] - (2.0 - 2.0 * cos((k + 1) * M_PI / (n + 1)))));
  /* random symmetric: trace / Frobenius invariants, Lower vs Upper */
  unsigned sd = 919;
  rnd_fill(a, (size_t)n * n, &sd);
  double tr = 0, fr = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < j; ++i) a[i + (size_t)j * n] = a[j + (size_t)i * n];
  for (int j = 0; j < n; ++j) {
    tr += a[j + (size_t)j * n];
    for (int i = 0; i < n; ++i) fr += a[i + (size_t)j * n] * a[i + (size_t)j * n];
  }
  dplasma_desc_set_lapack(A, a, n);
  CHECK(dplasma_dheev(ctx, dplasmaNoVec, dplasmaLower, A, W, NULL) == 0, "dheev L: %s", dplasma_last_error());
  dplasma_desc_get_lapack(W, w, n);
  dplasma_desc_set_lapack(A, a, n);
  CHECK(dplasma_dheev(ctx, dplasmaNoVec, dplasmaUpper, A, W, NULL) == 0, "dheev U: %s", dplasma_last_error());
  dplasma_desc_get_lapack(W, w2, n);
  double s1 = 0, s2 = 0, lu = 0, wmax = 0;
  int sorted = 1;
  for (int k = 0; k < n; ++k) {
    s1 += w[k], s2 += w[k] * w[k];
    lu = fmax(lu, fabs(w[k] - w2[k]));
    wmax = fmax(wmax, fabs(w[k]));
    if (k && w[k] < w[k - 1]) sorted = 0;
  }
  printf("dheev n=%d nb=%d: Laplacian max err %.2e  random: |sum l - tr| %.2e  |sum l^2 - ||A||_F^2|/||A||_F^2 %.2e  L vs U %.2e\n",
         n, nb, el, fabs(s1 - tr) / (n * wmax), fabs(s2 - fr) / fr, lu / wmax);
  CHECK(el < 1e-12 && fabs(s1 - tr) / (n * wmax) < 1e-13 && fabs(s2 - fr) / fr < 1e-12 && lu / wmax < 1e-12 && sorted,
        "dheev residuals");
  /* complex Hermitian */
  {
    const int nz = 300, nbz = 48;
    dplasma_desc_t *Z = dmat(ctx, dplasmaComplexDouble, nbz, nz, nz), *Wz = dmat(ctx, dplasmaRealDouble, nbz, nz, 1);
    double complex *z = malloc(sizeof(double complex) * nz * nz);
    double *re = malloc(sizeof(double) * 2 * nz * nz), *wz = malloc(sizeof(double) * nz);
    rnd_fill(re, (size_t)2 * nz * nz, &sd);
    for (int j = 0; j < nz; ++j)
      for (int i = 0; i < nz; ++i) z[i + (size_t)j * nz] = re[2 * (i + (size_t)j * nz)] + I * re[2 * (i + (size_t)j * nz) + 1];
    double trz = 0, frz = 0;
    for (int j = 0; j < nz; ++j) {
      z[j + (size_t)j * nz] = creal(z[j + (size_t)j * nz]);
      for (int i = 0; i < j; ++i) z[i + (size_t)j * nz] = conj(z[j + (size_t)i * nz]);
    }
    for (int j = 0; j < nz; ++j) {
      trz += creal(z[j + (size_t)j * nz]);
      for (int i = 0; i < nz; ++i) frz += creal(z[i + (size_t)j * nz] * conj(z[i + (size_t)j * nz]));
    }
    dplasma_desc_set_lapack(Z, z, nz);
    CHECK(dplasma_zheev(ctx, dplasmaNoVec, dplasmaLower, Z, Wz, NULL) == 0, "zheev: %s", dplasma_last_error());
    dplasma_desc_get_lapack(Wz, wz, nz);
    double t1 = 0, t2 = 0, wm = 0;
    for (int k = 0; k < nz; ++k) t1 += wz[k], t2 += wz[k] * wz[k], wm = fmax(wm, fabs(wz[k]));
    printf("zheev n=%d: |sum l - tr| %.2e  |sum l^2 - ||A||_F^2|/||A||_F^2 %.2e\n", nz, fabs(t1 - trz) / (nz * wm),
           fabs(t2 - frz) / frz);
    CHECK(fabs(t1 - trz) / (nz * wm) < 1e-13 && fabs(t2 - frz) / frz < 1e-12, "zheev invariants");
    free(z), free(re), free(wz);
    dplasma_desc_destroy(Z), dplasma_desc_destroy(Wz);
  }
  /* hbrdt on a band descriptor ((b+1) x n, lower band storage of a random symmetric band matrix) */
  {
    const int b = 16, nn = 400;
    dplasma_desc_t *Bd = dmat(ctx, dplasmaRealDouble, 64, b + 1, nn);
    double *ab = malloc(sizeof(double) * (b + 1) * nn), *out = malloc(sizeof(double) * (b + 1) * nn);
    rnd_fill(ab, (size_t)(b + 1) * nn, &sd);
    for (int j = 0; j < nn; ++j)
      for (int r = 0; r <= b; ++r)
        if (j + r >= nn) ab[r + (size_t)j * (b + 1)] = 0;
    double tb = 0, fb = 0;
    for (int j = 0; j < nn; ++j) {
      tb += ab[(size_t)j * (b + 1)];
      fb += ab[(size_t)j * (b + 1)] * ab[(size_t)j * (b + 1)];
      for (int r = 1; r <= b; ++r) fb += 2 * ab[r + (size_t)j * (b + 1)] * ab[r + (size_t)j * (b + 1)];
    }
    dplasma_desc_set_lapack(Bd, ab, b + 1);
    CHECK(dplasma_dhbrdt(ctx, Bd) == 0, "dhbrdt: %s", dplasma_last_error());
    dplasma_desc_get_lapack(Bd, out, b + 1);
    double td = 0, fd = 0, rest = 0;
    for (int j = 0; j < nn; ++j) {
      td += out[(size_t)j * (b + 1)];
      fd += out[(size_t)j * (b + 1)] * out[(size_t)j * (b + 1)];
      if (j + 1 < nn) fd += 2 * out[1 + (size_t)j * (b + 1)] * out[1 + (size_t)j * (b + 1)];
      for (int r = 2; r <= b; ++r) rest = fmax(rest, fabs(out[r + (size_t)j * (b + 1)]));
    }
    printf("dhbrdt b=%d n=%d: |trace d - trace| %.2e  |fro(d,e)^2 - fro^2|/fro^2 %.2e  rows >= 2 max %.1e\n", b, nn,
           fabs(td - tb), fabs(fd - fb) / fb, rest);
    CHECK(fabs(td - tb) < 1e-10 && fabs(fd - fb) / fb < 1e-12 && rest == 0, "hbrdt invariants");
    free(ab), free(out);
    dplasma_desc_destroy(Bd);
  }
  free(a), free(w), free(w2);
  dplasma_desc_destroy(A), dplasma_desc_destroy(W);
}

/* general -> upper band bidiagonal natively (gebrd_ge2gb; ge2gbx with flat native trees gives the same band): the
 * band keeps the Frobenius norm and holds nothing outside its nb + 1 diagonals; A and the band are dumped under
 * DPLASMA_TEST_DUMP for tests/test_capi.py to compare singular values with numpy */
static void test_ge2gb(dplasma_context_t *ctx) {
  const int m = 600, n = 400, nb = 64, ib = 16;
  const int mt = (m + nb - 1) / nb, nt = (n + nb - 1) / nb;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, m, n), *Bd = dmat(ctx, dplasmaRealDouble, nb, nb + 1, n);
  dplasma_desc_t *B2 = dmat(ctx, dplasmaRealDouble, nb, nb + 1, n);
  dplasma_desc_t *TS0 = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  dplasma_desc_t *TS = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, ib, nb, mt * ib, nt * nb, 1, 1, dplasmaUpperLower);
  CHECK(A && Bd && B2 && TS0 && TS, "ge2gb descriptors: %s", dplasma_last_error());
  double *a = malloc(sizeof(double) * m * n), *band = malloc(sizeof(double) * (nb + 1) * n);
  double *band2 = malloc(sizeof(double) * (nb + 1) * n);
  unsigned sd = 4242;
  rnd_fill(a, (size_t)m * n, &sd);
  double fa = 0;
  for (size_t e = 0; e < (size_t)m * n; ++e) fa += a[e] * a[e];
  dplasma_desc_set_lapack(A, a, m);
  CHECK(dplasma_dgebrd_ge2gb(ctx, ib, A, Bd) == 0, "dgebrd_ge2gb: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Bd, band, nb + 1);
  dplasma_qrtree_t tq, tl;
  memset(&tq, 0, sizeof tq), memset(&tl, 0, sizeof tl);
  CHECK(dplasma_hqr_init(&tq, dplasmaNoTrans, A, DPLASMA_FLAT_TREE, DPLASMA_FLAT_TREE, mt, 1, 0, 0) == 0 &&
        dplasma_hqr_init(&tl, dplasmaTrans, A, DPLASMA_FLAT_TREE, DPLASMA_FLAT_TREE, nt, 1, 0, 0) == 0, "flat trees: %s",
        dplasma_last_error());
  dplasma_desc_set_lapack(A, a, m);
  CHECK(dplasma_dgebrd_ge2gbx(ctx, ib, NULL, &tq, &tl, A, TS0, NULL, TS, NULL, B2) == 0, "dgebrd_ge2gbx: %s",
        dplasma_last_error());
  dplasma_desc_get_lapack(B2, band2, nb + 1);
  double fb = 0, dx = 0;
  for (int j = 0; j < n; ++j)
    for (int r = 0; r <= nb; ++r) {
      const double x = band[r + (size_t)j * (nb + 1)];
      fb += x * x;
      dx = fmax(dx, fabs(x - band2[r + (size_t)j * (nb + 1)]));
    }
  const char *dump = getenv("DPLASMA_TEST_DUMP");
  if (dump) {
    char path[512];
    snprintf(path, sizeof path, "%s/ge2gb_a.bin", dump);
    FILE *fp = fopen(path, "wb");
    if (fp) fwrite(a, sizeof(double), (size_t)m * n, fp), fclose(fp);
    snprintf(path, sizeof path, "%s/ge2gb_band.bin", dump);
    fp = fopen(path, "wb");
    if (fp) fwrite(band, sizeof(double), (size_t)(nb + 1) * n, fp), fclose(fp);
  }
  printf("dgebrd_ge2gb %dx%d nb=%d: | ||band||_F^2 - ||A||_F^2 | / ||A||_F^2 %.2e  ge2gbx (flat trees) vs ge2gb %.1e\n", m, n,
         nb, fabs(fb - fa) / fa, dx);
  CHECK(fabs(fb - fa) / fa < 1e-12 && dx == 0, "ge2gb band");
  dplasma_hqr_finalize(&tq), dplasma_hqr_finalize(&tl);
  free(a), free(band), free(band2);
  dplasma_desc_destroy(A), dplasma_desc_destroy(Bd), dplasma_desc_destroy(B2), dplasma_desc_destroy(TS0);
  dplasma_desc_destroy(TS);
}

/* trtri / lauum / potri / poinv natively: A := inv(A) checked as ||A0 inv(A) - I||; lauum against host
   L^T L; her2k / syr2k against host rank-2k; the alias entry points (ptgpanel on 1x1, potrf_rec). */
static void test_inverse_family(dplasma_context_t *ctx) {
  const int n = 700, nb = 128;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  double *A0 = malloc(sizeof(double) * n * n), *X = malloc(sizeof(double) * n * n);
  CHECK(dplasma_dplghe(ctx, (double)n, dplasmaUpperLower, A, 77) == 0, "dplghe: %s", dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, A0, n) == 0, "get A0");
  CHECK(dplasma_dpoinv(ctx, dplasmaLower, A) == 0, "dpoinv: %s", dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, X, n) == 0, "get X");
  for (int j = 0; j < n; ++j)   /* symmetric inverse from its lower triangle */
    for (int i = 0; i < j; ++i) X[i + (size_t)j * n] = X[j + (size_t)i * n];
  double err = 0;
  for (int j = 0; j < n; j += 7)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += A0[i + (size_t)k * n] * X[k + (size_t)j * n];
      err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
    }
  CHECK(err < 1e-10, "dpoinv ||A inv(A) - I|| %.3e", err);
  /* trtri of a unit upper triangle: T inv(T) = I on the upper part */
  CHECK(dplasma_dplrnt(ctx, 0, A, 5) == 0, "dplrnt");
  /* small off-diagonal entries: a random unit triangle of order 700 has an exponentially large inverse */
  CHECK(dplasma_dlascal(ctx, dplasmaUpperLower, 0.02, A) == 0, "dlascal");
  CHECK(dplasma_desc_get_lapack(A, A0, n) == 0, "get T0");
  CHECK(dplasma_dtrtri(ctx, dplasmaUpper, dplasmaUnit, A) == 0, "dtrtri: %s", dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, X, n) == 0, "get inv");
  err = 0;
  for (int j = 0; j < n; j += 5)
    for (int i = 0; i <= j; ++i) {
      double s = 0;
      for (int k = i; k <= j; ++k)
        s += (k == i ? 1.0 : A0[i + (size_t)k * n]) * (k == j ? 1.0 : X[k + (size_t)j * n]);
      err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
    }
  CHECK(err < 1e-12, "dtrtri unit upper error %.3e", err);
  /* lauum lower: A := L^T L */
  CHECK(dplasma_dplrnt(ctx, 0, A, 9) == 0, "dplrnt");
  CHECK(dplasma_desc_get_lapack(A, A0, n) == 0, "get L0");
  CHECK(dplasma_dlauum(ctx, dplasmaLower, A) == 0, "dlauum: %s", dplasma_last_error());
  CHECK(dplasma_desc_get_lapack(A, X, n) == 0, "get LtL");
  err = 0;
  double nrm = 0;
  for (int j = 0; j < n; j += 3)
    for (int i = j; i < n; ++i) {
      double s = 0;
      for (int k = i; k < n; ++k) s += A0[k + (size_t)i * n] * A0[k + (size_t)j * n];
      err = fmax(err, fabs(X[i + (size_t)j * n] - s));
      nrm = fmax(nrm, fabs(s));
    }
  CHECK(err < 1e-13 * nrm * n, "dlauum error %.3e", err / nrm);
  dplasma_desc_destroy(A);
  free(A0);
  free(X);
}

static void test_rank_2k(dplasma_context_t *ctx) {
  const int n = 300, k = 200, nb = 128;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, k), *B = dmat(ctx, dplasmaRealDouble, nb, n, k);
  dplasma_desc_t *C = dmat(ctx, dplasmaRealDouble, nb, n, n);
  double *a = malloc(sizeof(double) * n * k), *b = malloc(sizeof(double) * n * k);
  double *c0 = malloc(sizeof(double) * n * n), *c1 = malloc(sizeof(double) * n * n);
  dplasma_dplrnt(ctx, 0, A, 1);
  dplasma_dplrnt(ctx, 0, B, 2);
  dplasma_dplrnt(ctx, 0, C, 3);
  dplasma_desc_get_lapack(A, a, n);
  dplasma_desc_get_lapack(B, b, n);
  dplasma_desc_get_lapack(C, c0, n);
  CHECK(dplasma_dsyr2k(ctx, dplasmaUpper, dplasmaNoTrans, 0.7, A, B, -0.3, C) == 0, "dsyr2k: %s",
        dplasma_last_error());
  dplasma_desc_get_lapack(C, c1, n);
  double err = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i <= j; ++i) {
      double s = 0;
      for (int q = 0; q < k; ++q) s += a[i + (size_t)q * n] * b[j + (size_t)q * n] + b[i + (size_t)q * n] * a[j + (size_t)q * n];
      err = fmax(err, fabs(c1[i + (size_t)j * n] - (0.7 * s - 0.3 * c0[i + (size_t)j * n])));
    }
  CHECK(err < 1e-11, "dsyr2k error %.3e", err);
  dplasma_desc_destroy(A);
  dplasma_desc_destroy(B);
  dplasma_desc_destroy(C);
  /* zher2k: C = alpha A B^H + conj(alpha) B A^H + beta C, real diagonal */
  dplasma_desc_t *Z = dmat(ctx, dplasmaComplexDouble, nb, n, k), *Y = dmat(ctx, dplasmaComplexDouble, nb, n, k);
  dplasma_desc_t *W = dmat(ctx, dplasmaComplexDouble, nb, n, n);
  double complex *z = malloc(sizeof(double complex) * n * k), *y = malloc(sizeof(double complex) * n * k);
  double complex *w0 = malloc(sizeof(double complex) * n * n), *w1 = malloc(sizeof(double complex) * n * n);
  dplasma_zplrnt(ctx, 0, Z, 4);
  dplasma_zplrnt(ctx, 0, Y, 5);
  dplasma_zplghe(ctx, 1.0, dplasmaUpperLower, W, 6);
  dplasma_desc_get_lapack(Z, z, n);
  dplasma_desc_get_lapack(Y, y, n);
  dplasma_desc_get_lapack(W, w0, n);
  const double complex al = 0.5 + 0.25 * I;
  CHECK(dplasma_zher2k(ctx, dplasmaLower, dplasmaNoTrans, al, Z, Y, 0.5, W) == 0, "zher2k: %s", dplasma_last_error());
  dplasma_desc_get_lapack(W, w1, n);
  err = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) {
      double complex s = 0;
      for (int q = 0; q < k; ++q)
        s += al * z[i + (size_t)q * n] * conj(y[j + (size_t)q * n]) + conj(al) * y[i + (size_t)q * n] * conj(z[j + (size_t)q * n]);
      err = fmax(err, cabs(w1[i + (size_t)j * n] - (s + 0.5 * w0[i + (size_t)j * n])));
    }
  CHECK(err < 1e-11, "zher2k error %.3e", err);
  for (int i = 0; i < n; ++i) CHECK(cimag(w1[i + (size_t)i * n]) == 0.0, "zher2k diagonal imaginary part");
  dplasma_desc_destroy(Z);
  dplasma_desc_destroy(Y);
  dplasma_desc_destroy(W);
  free(a); free(b); free(c0); free(c1); free(z); free(y); free(w0); free(w1);
}

static void test_aliases(dplasma_context_t *ctx) {
  const int n = 512, nb = 128;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, 1, nb, 1, n, 1, 1);
  CHECK(A && IP, "alias descriptors: %s", dplasma_last_error());
  dplasma_dplrnt(ctx, 0, A, 8);
  CHECK(dplasma_dgetrf_ptgpanel(ctx, A, IP) == 0, "dgetrf_ptgpanel (1x1 native): %s", dplasma_last_error());
  dplasma_dplghe(ctx, (double)n, dplasmaLower, A, 3);
  CHECK(dplasma_dpotrf_rec(ctx, dplasmaLower, A, 64) == 0, "dpotrf_rec (native): %s", dplasma_last_error());
  dplasma_desc_destroy(A);
  dplasma_desc_destroy(IP);
}

/* dgeru / zgerc natively (a K = 1 GEMM): A := alpha x y^T + A, A := alpha x y^H + A, ragged 300 x 200, nb 128 */
static void test_ger(dplasma_context_t *ctx) {
  const int M = 300, N = 200, nb = 128;
  dplasma_desc_t *X = dmat(ctx, dplasmaRealDouble, nb, M, 1), *Y = dmat(ctx, dplasmaRealDouble, nb, N, 1);
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, M, N);
  dplasma_dplrnt(ctx, 0, X, 11);
  dplasma_dplrnt(ctx, 0, Y, 12);
  dplasma_dplrnt(ctx, 0, A, 13);
  double *x = malloc(sizeof(double) * M), *y = malloc(sizeof(double) * N);
  double *a = malloc(sizeof(double) * M * N), *r = malloc(sizeof(double) * M * N);
  dplasma_desc_get_lapack(X, x, M);
  dplasma_desc_get_lapack(Y, y, N);
  dplasma_desc_get_lapack(A, a, M);
  CHECK(dplasma_dgeru(ctx, 0.75, X, Y, A) == 0, "dgeru: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, r, M);
  double err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) err = fmax(err, fabs(a[i + (size_t)j * M] + 0.75 * x[i] * y[j] - r[i + (size_t)j * M]));
  printf("dgeru %dx%d max error %.3e\n", M, N, err);
  CHECK(err < 1e-13, "dgeru error %.3e", err);
  free(x), free(y), free(a), free(r);
  dplasma_desc_destroy(X), dplasma_desc_destroy(Y), dplasma_desc_destroy(A);
  /* zgerc: the conjugate of y */
  dplasma_desc_t *Xz = dmat(ctx, dplasmaComplexDouble, nb, M, 1), *Yz = dmat(ctx, dplasmaComplexDouble, nb, N, 1);
  dplasma_desc_t *Az = dmat(ctx, dplasmaComplexDouble, nb, M, N);
  dplasma_zplrnt(ctx, 0, Xz, 21);
  dplasma_zplrnt(ctx, 0, Yz, 22);
  dplasma_zplrnt(ctx, 0, Az, 23);
  double complex *xz = malloc(sizeof(double complex) * M), *yz = malloc(sizeof(double complex) * N);
  double complex *az = malloc(sizeof(double complex) * M * N), *rz = malloc(sizeof(double complex) * M * N);
  dplasma_desc_get_lapack(Xz, xz, M);
  dplasma_desc_get_lapack(Yz, yz, N);
  dplasma_desc_get_lapack(Az, az, M);
  const double complex alpha = 0.5 - 0.25 * _Complex_I;
  CHECK(dplasma_zgerc(ctx, alpha, Xz, Yz, Az) == 0, "zgerc: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Az, rz, M);
  err = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i)
      err = fmax(err, cabs(az[i + (size_t)j * M] + alpha * xz[i] * conj(yz[j]) - rz[i + (size_t)j * M]));
  printf("zgerc %dx%d max error %.3e\n", M, N, err);
  CHECK(err < 1e-13, "zgerc error %.3e", err);
  free(xz), free(yz), free(az), free(rz);
  dplasma_desc_destroy(Xz), dplasma_desc_destroy(Yz), dplasma_desc_destroy(Az);
}

/* dlaswp natively: the pivots of a getrf applied forward to a 700 x 9 matrix (vs the same swaps on the host),
 * then undone (inc = -1) back to the original */
static void test_laswp(dplasma_context_t *ctx) {
  const int n = 700, nb = 256, nc = 9;
  dplasma_desc_t *G = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nc);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, 1, nb, 1, n, 1, 1);
  double *g = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nc), *r = malloc(sizeof(double) * n * nc);
  int *ipiv = malloc(sizeof(int) * n);
  unsigned sd = 77;
  rnd_fill(g, (size_t)n * n, &sd), rnd_fill(b, (size_t)n * nc, &sd);
  dplasma_desc_set_lapack(G, g, n);
  CHECK(dplasma_dgetrf_1d(ctx, G, IP) == 0, "laswp: getrf %s", dplasma_last_error());
  dplasma_desc_get_lapack(IP, ipiv, 1);
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dlaswp(ctx, B, IP, 1) == 0, "dlaswp: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, r, n);
  for (int i = 0; i < n; ++i) {   /* host reference: LAPACK dlaswp, k1 = 1 .. n, incx = 1 */
    const int p = ipiv[i] - 1;
    if (p != i)
      for (int c = 0; c < nc; ++c) {
        const double t = b[i + (size_t)c * n];
        b[i + (size_t)c * n] = b[p + (size_t)c * n];
        b[p + (size_t)c * n] = t;
      }
  }
  double err = 0;
  for (size_t e = 0; e < (size_t)n * nc; ++e) err = fmax(err, fabs(r[e] - b[e]));
  CHECK(err == 0.0, "dlaswp forward differs (%.3e)", err);
  CHECK(dplasma_dlaswp(ctx, B, IP, -1) == 0, "dlaswp back: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, r, n);
  unsigned sd2 = 77;
  rnd_fill(g, (size_t)n * n, &sd2), rnd_fill(b, (size_t)n * nc, &sd2);   /* the original B again */
  err = 0;
  for (size_t e = 0; e < (size_t)n * nc; ++e) err = fmax(err, fabs(r[e] - b[e]));
  printf("dlaswp %d x %d forward exact, undone: max diff %.3e\n", n, nc, err);
  CHECK(err == 0.0, "dlaswp inc -1 did not undo (%.3e)", err);
  free(g), free(b), free(r), free(ipiv);
  dplasma_desc_destroy(G), dplasma_desc_destroy(B), dplasma_desc_destroy(IP);
}

/* dlanm2 natively: ||u v^T||_2 = ||u|| ||v|| (the rank-one matrix built with dgeru on a zero matrix), and a
 * diagonal matrix diag(3n, 2, .., n) whose 2-norm is 3n (a separated top singular value: fast convergence) */
static void test_lanm2(dplasma_context_t *ctx) {
  const int M = 300, N = 200, nb = 128;
  dplasma_desc_t *X = dmat(ctx, dplasmaRealDouble, nb, M, 1), *Y = dmat(ctx, dplasmaRealDouble, nb, N, 1);
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, M, N);
  dplasma_dplrnt(ctx, 0, X, 41);
  dplasma_dplrnt(ctx, 0, Y, 42);
  dplasma_dlaset(ctx, dplasmaUpperLower, 0.0, 0.0, A);
  CHECK(dplasma_dgeru(ctx, 1.0, X, Y, A) == 0, "lanm2: dgeru %s", dplasma_last_error());
  const double nu = dplasma_dlange(ctx, dplasmaFrobeniusNorm, X), nv = dplasma_dlange(ctx, dplasmaFrobeniusNorm, Y);
  int info = 0;
  const double e = dplasma_dlanm2(ctx, A, &info);
  printf("dlanm2 rank-one %dx%d: %.15g vs %.15g (info %d)\n", M, N, e, nu * nv, info);
  CHECK(fabs(e - nu * nv) <= 1e-12 * nu * nv && info > 0, "dlanm2 rank one: %.15g vs %.15g (info %d, %s)", e,
        nu * nv, info, dplasma_last_error());
  const int n = 257;
  dplasma_desc_t *D = dmat(ctx, dplasmaRealDouble, nb, n, n);
  double *d = calloc((size_t)n * n, sizeof(double));
  for (int i = 0; i < n; ++i) d[i + (size_t)i * n] = i == 0 ? 3.0 * n : i + 1;
  dplasma_desc_set_lapack(D, d, n);
  const double e2 = dplasma_dlanm2(ctx, D, &info);
  printf("dlanm2 diag(3n, 2..%d): %.12g (info %d)\n", n, e2, info);
  CHECK(fabs(e2 - 3.0 * n) <= 1e-8 * n, "dlanm2 diagonal: %.12g vs %d", e2, 3 * n);
  free(d);
  dplasma_desc_destroy(X), dplasma_desc_destroy(Y), dplasma_desc_destroy(A), dplasma_desc_destroy(D);
}

/* the solve-side EXT ops natively: dtrsmpl_ptgpanel (B := L^-1 P B with the getrf_1d factors, checked as
 * L Y = P B on the host), dtrdsm (B := D^-1 B), dtrmdm (strict lower part := L D^-1) and dprint */
static void test_trsmpl_diag(dplasma_context_t *ctx) {
  const int n = 600, nb = 256, nc = 7;
  dplasma_desc_t *G = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nc);
  dplasma_desc_t *IP = dplasma_desc_ipiv(ctx, 1, nb, 1, n, 1, 1);
  double *g = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nc), *y = malloc(sizeof(double) * n * nc);
  int *ipiv = malloc(sizeof(int) * n);
  unsigned sd = 91;
  rnd_fill(g, (size_t)n * n, &sd), rnd_fill(b, (size_t)n * nc, &sd);
  dplasma_desc_set_lapack(G, g, n);
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dgetrf_1d(ctx, G, IP) == 0, "trsmpl: getrf %s", dplasma_last_error());
  CHECK(dplasma_dtrsmpl_ptgpanel(ctx, G, IP, B) == 0, "dtrsmpl_ptgpanel: %s", dplasma_last_error());
  dplasma_desc_get_lapack(G, g, n);
  dplasma_desc_get_lapack(IP, ipiv, 1);
  dplasma_desc_get_lapack(B, y, n);
  for (int i = 0; i < n; ++i) {   /* P b on the host */
    const int p = ipiv[i] - 1;
    if (p != i)
      for (int c = 0; c < nc; ++c) {
        const double t = b[i + (size_t)c * n];
        b[i + (size_t)c * n] = b[p + (size_t)c * n];
        b[p + (size_t)c * n] = t;
      }
  }
  double err = 0, scale = 0;
  for (int c = 0; c < nc; ++c)
    for (int i = 0; i < n; ++i) {
      double s = y[i + (size_t)c * n];   /* unit diagonal */
      for (int k = 0; k < i; ++k) s += g[i + (size_t)k * n] * y[k + (size_t)c * n];
      err = fmax(err, fabs(s - b[i + (size_t)c * n]));
      scale = fmax(scale, fabs(b[i + (size_t)c * n]));
    }
  printf("dtrsmpl_ptgpanel %d x %d: max |L Y - P B| %.3e\n", n, nc, err);
  CHECK(err < 1e-11 * fmax(1.0, scale) * n, "dtrsmpl_ptgpanel error %.3e", err);
  /* trdsm / trmdm on a matrix with a nonzero diagonal */
  for (int i = 0; i < n; ++i) g[i + (size_t)i * n] = 2.0 + 0.01 * i;
  rnd_fill(b, (size_t)n * nc, &sd);
  dplasma_desc_set_lapack(G, g, n);
  dplasma_desc_set_lapack(B, b, n);
  CHECK(dplasma_dtrdsm(ctx, G, B) == 0, "dtrdsm: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, y, n);
  err = 0;
  for (int c = 0; c < nc; ++c)
    for (int i = 0; i < n; ++i) err = fmax(err, fabs(y[i + (size_t)c * n] - b[i + (size_t)c * n] / g[i + (size_t)i * n]));
  printf("dtrdsm %d x %d: max diff %.3e\n", n, nc, err);
  CHECK(err < 1e-15, "dtrdsm differs (%.3e)", err);
  double *r = malloc(sizeof(double) * n * n);
  CHECK(dplasma_dtrmdm(ctx, G) == 0, "dtrmdm: %s", dplasma_last_error());
  dplasma_desc_get_lapack(G, r, n);
  err = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      const double want = i > j ? g[i + (size_t)j * n] / g[j + (size_t)j * n] : g[i + (size_t)j * n];
      err = fmax(err, fabs(r[i + (size_t)j * n] - want));
    }
  printf("dtrmdm %d x %d: max diff %.3e\n", n, n, err);
  CHECK(err < 1e-15, "dtrmdm differs (%.3e)", err);
  dplasma_desc_t *S = dmat(ctx, dplasmaRealDouble, 2, 3, 3);
  double s9[9] = {1, 2, 3, 4, 5, 6, 7, 8, 9};
  dplasma_desc_set_lapack(S, s9, 3);
  CHECK(dplasma_dprint(ctx, dplasmaLower, S) == 0, "dprint: %s", dplasma_last_error());
  free(g), free(b), free(y), free(r), free(ipiv);
  dplasma_desc_destroy(G), dplasma_desc_destroy(B), dplasma_desc_destroy(IP), dplasma_desc_destroy(S);
}

/* LDL^H without pivoting natively: dhetrf + dhetrs on a symmetric diagonally dominant matrix (plgsy) and zhetrf +
 * zhetrs on a Hermitian one (plghe), the residual checked against the host copy of the full matrix */
static void test_hetrf(dplasma_context_t *ctx) {
  const int n = 600, nb = 256, nrhs = 3;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_dplgsy(ctx, (double)n, dplasmaUpperLower, A, 51);
  dplasma_dplrnt(ctx, 0, B, 52);
  double *a = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  dplasma_desc_get_lapack(A, a, n);
  dplasma_desc_get_lapack(B, b, n);
  int info = dplasma_dhetrf(ctx, A);
  CHECK(info == 0, "dhetrf info %d (%s)", info, dplasma_last_error());
  CHECK(dplasma_dhetrs(ctx, dplasmaLower, A, B, NULL, 0) == 0, "dhetrs: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, x, n);
  double err = 0, bn = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)c * n];
      err = fmax(err, fabs(s - b[i + (size_t)c * n]));
      bn = fmax(bn, fabs(b[i + (size_t)c * n]));
    }
  printf("dhetrf + dhetrs n=%d nb=%d: ||Ax-b||/||b|| %.3e\n", n, nb, err / bn);
  CHECK(err / bn < 1e-10, "dhetrf/dhetrs residual %.3e", err / bn);
  free(a), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
  dplasma_desc_t *Az = dmat(ctx, dplasmaComplexDouble, nb, n, n), *Bz = dmat(ctx, dplasmaComplexDouble, nb, n, nrhs);
  dplasma_zplghe(ctx, (double)n, dplasmaUpperLower, Az, 61);
  dplasma_zplrnt(ctx, 0, Bz, 62);
  double complex *az = malloc(sizeof(double complex) * n * n), *bz = malloc(sizeof(double complex) * n * nrhs);
  double complex *xz = malloc(sizeof(double complex) * n * nrhs);
  dplasma_desc_get_lapack(Az, az, n);
  dplasma_desc_get_lapack(Bz, bz, n);
  info = dplasma_zhetrf(ctx, Az);
  CHECK(info == 0, "zhetrf info %d (%s)", info, dplasma_last_error());
  CHECK(dplasma_zhetrs(ctx, dplasmaLower, Az, Bz, NULL, 0) == 0, "zhetrs: %s", dplasma_last_error());
  dplasma_desc_get_lapack(Bz, xz, n);
  err = 0, bn = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double complex s = 0;
      for (int k = 0; k < n; ++k) s += az[i + (size_t)k * n] * xz[k + (size_t)c * n];
      err = fmax(err, cabs(s - bz[i + (size_t)c * n]));
      bn = fmax(bn, cabs(bz[i + (size_t)c * n]));
    }
  printf("zhetrf + zhetrs n=%d nb=%d: ||Ax-b||/||b|| %.3e\n", n, nb, err / bn);
  CHECK(err / bn < 1e-10, "zhetrf/zhetrs residual %.3e", err / bn);
  free(az), free(bz), free(xz);
  dplasma_desc_destroy(Az), dplasma_desc_destroy(Bz);
}

/* dlatms natively: ||A||_F^2 = sum D(i)^2 (unitary invariance), and the symmetric form is symmetric */
static void test_latms(dplasma_context_t *ctx) {
  const int n = 400, nb = 128;
  const double cond = 1e3, tmp = 1.0 / cond, alp = (1.0 - tmp) / (n - 1);
  double f2 = 0;
  for (int i = 0; i < n; ++i) {
    const double d = i == 0 ? 1.0 : (n - i - 1) * alp + tmp;
    f2 += d * d;
  }
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  CHECK(dplasma_dlatms(ctx, dplasmaGeneral, cond, A, 3872) == 0, "dlatms general: %s", dplasma_last_error());
  const double fg = dplasma_dlange(ctx, dplasmaFrobeniusNorm, A);
  CHECK(dplasma_dlatms(ctx, dplasmaSymmetric, cond, A, 3872) == 0, "dlatms symmetric: %s", dplasma_last_error());
  const double fs = dplasma_dlange(ctx, dplasmaFrobeniusNorm, A);
  double *a = malloc(sizeof(double) * n * n);
  dplasma_desc_get_lapack(A, a, n);
  double asym = 0, amax = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      asym = fmax(asym, fabs(a[i + (size_t)j * n] - a[j + (size_t)i * n]));
      amax = fmax(amax, fabs(a[i + (size_t)j * n]));
    }
  printf("dlatms n=%d cond=%g: ||A||_F %.15g / %.15g vs %.15g, symmetric form |A - A^T| %.3e\n", n, cond, fg, fs,
         sqrt(f2), asym);
  CHECK(fabs(fg - sqrt(f2)) < 1e-12 * sqrt(f2) && fabs(fs - sqrt(f2)) < 1e-12 * sqrt(f2), "dlatms Frobenius");
  CHECK(asym < 1e-13 * fmax(amax, 1e-300) * n, "dlatms symmetric form not symmetric (%.3e)", asym);
  free(a);
  dplasma_desc_destroy(A);
}

/* dposv on a matrix that is not positive definite: info > 0 and B left unchanged (zposv_wrapper.c runs potrs
 * only when info == 0) */
static void test_posv_not_spd(dplasma_context_t *ctx) {
  const int n = 300, nb = 128, nrhs = 2;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_dplgsy(ctx, 0.0, dplasmaUpperLower, A, 71);   /* no diagonal bump: indefinite */
  dplasma_dplrnt(ctx, 0, B, 72);
  double *b = malloc(sizeof(double) * n * nrhs), *r = malloc(sizeof(double) * n * nrhs);
  dplasma_desc_get_lapack(B, b, n);
  const int info = dplasma_dposv(ctx, dplasmaLower, A, B);
  dplasma_desc_get_lapack(B, r, n);
  double d = 0;
  for (size_t e = 0; e < (size_t)n * nrhs; ++e) d = fmax(d, fabs(r[e] - b[e]));
  printf("dposv on an indefinite matrix: info %d, B changed by %.3e\n", info, d);
  CHECK(info > 0 && d == 0.0, "dposv indefinite: info %d, B changed by %.3e", info, d);
  free(b), free(r);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

/* dpltmg natively (closed-form types): hilb / minij element values, hadamard H H^T = n I, a random-vector type
 * (house) refused with -2 */
static void test_pltmg(dplasma_context_t *ctx) {
  const int n = 256, nb = 96;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n);
  double *a = malloc(sizeof(double) * n * n);
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixHilb, A, 3872) == 0, "dpltmg hilb: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  double err = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) err = fmax(err, fabs(a[i + (size_t)j * n] - 1.0 / (i + j + 1.0)));
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixMinij, A, 3872) == 0, "dpltmg minij: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) err = fmax(err, fabs(a[i + (size_t)j * n] - (double)(i < j ? i + 1 : j + 1)));
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixHadamard, A, 3872) == 0, "dpltmg hadamard: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  double orth = 0;
  for (int j = 0; j < n; j += 17)
    for (int i = 0; i < n; i += 13) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * a[j + (size_t)k * n];
      orth = fmax(orth, fabs(s - (i == j ? n : 0)));
    }
  /* house: a symmetric orthogonal reflector, H H = I */
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixHouse, A, 3872) == 0, "dpltmg house: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  double hh = 0;
  for (int j = 0; j < n; j += 11)
    for (int i = 0; i < n; i += 7) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * a[k + (size_t)j * n];
      hh = fmax(hh, fabs(s - (i == j ? 1.0 : 0.0)));
      hh = fmax(hh, fabs(a[i + (size_t)j * n] - a[j + (size_t)i * n]));
    }
  /* circul: A(i, j) = A(i + 1, j + 1) (mod n) */
  CHECK(dplasma_dpltmg(ctx, dplasmaMatrixCircul, A, 3872) == 0, "dpltmg circul: %s", dplasma_last_error());
  dplasma_desc_get_lapack(A, a, n);
  double circ = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) circ = fmax(circ, fabs(a[i + (size_t)j * n] - a[(i + 1) % n + (size_t)((j + 1) % n) * n]));
  const int rx = dplasma_dpltmg(ctx, 6 /* toeppen: not in the reference */, A, 3872);
  printf("dpltmg hilb / minij max error %.3e, hadamard |H H^T - n I| %.3e, house |H H - I| %.3e, circulant %.3e, "
         "toeppen -> %d\n", err, orth, hh, circ, rx);
  CHECK(err == 0.0 && orth == 0.0 && hh < 1e-13 && circ == 0.0 && rx == -2, "dpltmg: err %.3e orth %.3e house %.3e "
        "circ %.3e toeppen %d", err, orth, hh, circ, rx);
  /* DPLASMA_TEST_DUMP=dir: every random-vector type (d and z) for tests/test_capi.py to compare with the Python layer */
  const char *dump = getenv("DPLASMA_TEST_DUMP");
  if (dump) {
    const int m2 = 40, n2 = 36, nb2 = 16;
    const int types[] = {2, 7, 9, 12, 14, 23, 27, 29, 42};
    for (int z = 0; z < 2; ++z) {
      dplasma_desc_t *B = dmat(ctx, z ? dplasmaComplexDouble : dplasmaRealDouble, nb2, m2, n2);
      double *b = malloc(sizeof(double) * 2 * m2 * n2);
      for (unsigned q = 0; q < sizeof types / sizeof types[0]; ++q) {
        const int r = z ? dplasma_zpltmg(ctx, types[q], B, 3872) : dplasma_dpltmg(ctx, types[q], B, 3872);
        CHECK(r == 0, "%cpltmg type %d: %d (%s)", z ? 'z' : 'd', types[q], r, dplasma_last_error());
        dplasma_desc_get_lapack(B, b, m2);
        char path[4096];
        snprintf(path, sizeof path, "%s/pltmg_%c_%d.bin", dump, z ? 'z' : 'd', types[q]);
        FILE *f = fopen(path, "wb");
        CHECK(f != NULL, "cannot write %s", path);
        fwrite(b, sizeof(double) * (z ? 2 : 1), (size_t)m2 * n2, f);
        fclose(f);
      }
      free(b);
      dplasma_desc_destroy(B);
    }
  }
  free(a);
  dplasma_desc_destroy(A);
}

/* random butterflies natively: hebut (A := U^T A U, U returned on the host), hetrf without pivoting on the
 * transformed matrix, hetrs with the butterfly (x = U (L D L^T)^-1 U^T b) -- the residual on the original A */
static void test_butterfly(dplasma_context_t *ctx) {
  const int n = 512, nb = 128, nrhs = 2, level = 2;
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, nb, n, n), *B = dmat(ctx, dplasmaRealDouble, nb, n, nrhs);
  dplasma_dplgsy(ctx, 1.0, dplasmaUpperLower, A, 81);   /* symmetric, small bump: indefinite */
  dplasma_dplrnt(ctx, 0, B, 82);
  double *a = malloc(sizeof(double) * n * n), *b = malloc(sizeof(double) * n * nrhs), *x = malloc(sizeof(double) * n * nrhs);
  dplasma_desc_get_lapack(A, a, n);
  dplasma_desc_get_lapack(B, b, n);
  double *U = NULL;
  CHECK(dplasma_dhebut(ctx, A, &U, level) == 0 && U != NULL, "dhebut: %s", dplasma_last_error());
  int info = dplasma_dhetrf(ctx, A);
  CHECK(info == 0, "dhetrf after hebut: info %d (%s)", info, dplasma_last_error());
  CHECK(dplasma_dhetrs(ctx, dplasmaLower, A, B, U, level) == 0, "dhetrs with butterfly: %s", dplasma_last_error());
  dplasma_desc_get_lapack(B, x, n);
  double err = 0, bn = 0, xn = 0;
  for (int c = 0; c < nrhs; ++c)
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += a[i + (size_t)k * n] * x[k + (size_t)c * n];
      err = fmax(err, fabs(s - b[i + (size_t)c * n]));
      bn = fmax(bn, fabs(b[i + (size_t)c * n]));
      xn = fmax(xn, fabs(x[i + (size_t)c * n]));
    }
  printf("dhebut + dhetrf + dhetrs (butterfly depth %d) n=%d: ||Ax-b||/||b|| %.3e (|x| %.3e)\n", level, n, err / bn, xn);
  CHECK(err / bn < 1e-8, "butterfly solve residual %.3e", err / bn);
  free(U), free(a), free(b), free(x);
  dplasma_desc_destroy(A), dplasma_desc_destroy(B);
}

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  signal(SIGSEGV, on_fault);
  dplasma_context_t *ctx = dplasma_init_native(0);
  if (!ctx) {
    printf("dplasma_init_native failed: %s\n", dplasma_last_error());
    return 2;
  }
  CHECK(dplasma_context_world(ctx) == 1 && dplasma_context_rank(ctx) == 0, "rank/world");
  printf("native context up\n");
  test_dpotrf_posv(ctx);
  test_dposv_one_tile(ctx);
  test_dgemm(ctx);
  test_dtrsm(ctx, dplasmaLeft, dplasmaLower, dplasmaNoTrans);
  test_dtrsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaTrans);
  test_dtrsm(ctx, dplasmaRight, dplasmaUpper, dplasmaNoTrans);
  test_dtrsm(ctx, dplasmaRight, dplasmaLower, dplasmaTrans);
  test_zpotrf_spotrf(ctx);
  test_rank_k(ctx);
  test_maps(ctx);
  test_norms(ctx);
  test_taskpools(ctx);
  test_dtrmm(ctx, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit);
  test_dtrmm(ctx, dplasmaLeft, dplasmaUpper, dplasmaTrans, dplasmaUnit);
  test_dtrmm(ctx, dplasmaRight, dplasmaUpper, dplasmaNoTrans, dplasmaUnit);
  test_dtrmm(ctx, dplasmaRight, dplasmaLower, dplasmaTrans, dplasmaNonUnit);
  test_symm_hemm(ctx);
  test_dgetrf(ctx);
  test_dgeqrf(ctx);
  test_dgetrf_nopiv(ctx);
  test_dgesv_incpiv(ctx);
  test_dgelqf(ctx);
  test_zgelqf(ctx);
  test_dgeqrf_param(ctx);
  test_dgelqf_param(ctx);
  test_dgetrf_qrf(ctx);
  test_dgetrf_qrf_criteria(ctx);
  test_heev(ctx);
  test_ge2gb(ctx);
  test_inverse_family(ctx);
  test_rank_2k(ctx);
  test_aliases(ctx);
  test_ger(ctx);
  test_laswp(ctx);
  test_lanm2(ctx);
  test_trsmpl_diag(ctx);
  test_hetrf(ctx);
  test_latms(ctx);
  test_posv_not_spd(ctx);
  test_pltmg(ctx);
  test_butterfly(ctx);
  /* a request outside the native engine's scope fails cleanly (heev computes eigenvalues only, as the reference) */
  dplasma_desc_t *A = dmat(ctx, dplasmaRealDouble, 64, 128, 128);
  CHECK(dplasma_dheev(ctx, dplasmaVec, dplasmaLower, A, A, NULL) != 0 && strstr(dplasma_last_error(), "NoVec") != NULL,
        "refused request: '%s'", dplasma_last_error());
  dplasma_desc_destroy(A);
  if (argc > 1 && atoi(argv[1]) > 0) bench(ctx, atoi(argv[1]));
  CHECK(dplasma_python_active() == 0, "the interpreter was started");
  dplasma_fini(ctx);
  if (fails)
    printf("native C ABI: %d FAILED\n", fails);
  else
    printf("native C ABI: all passed\n");
  return fails ? 1 : 0;
}
