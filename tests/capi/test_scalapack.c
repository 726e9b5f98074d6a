/* C ABI: taskpool lifecycle (dplasma_dpotrf_New / add / start / wait / _Destruct) on a descriptor over
 * caller-owned memory, then the ScaLAPACK F77 layer (BLACS shims, descinit_, pdpotrf_, pdgemm_,
 * pdtrsm_, pdgetrf_) on plain local arrays -- the flow of the reference's scalapack wrappers
 * (src/scalapack_wrappers) from a program that never touches Python.
 * usage: test_scalapack <gpus>   (gpus = 0: CPU path; the F77 arrays are host memory either way) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dplasma.h"

static int fail(const char *what) {
  fprintf(stderr, "FAIL %s: %s\n", what, dplasma_last_error());
  return 1;
}

static void spd(double *a, int n, int lda) {
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) a[i + (size_t)j * lda] = (i == j ? n : 0) + 1.0 / (1.0 + abs(i - j)) + 0.01 * sin(i + j);
}

/* max |L L^T - A| / max |A| over the lower triangle (L in the lower part of l) */
static double chol_res(const double *l, const double *a, int n, int lda) {
  double num = 0, den = 0;
  for (int j = 0; j < n; ++j)
    for (int i = j; i < n; ++i) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += l[i + (size_t)k * lda] * l[j + (size_t)k * lda];
      num = fmax(num, fabs(s - a[i + (size_t)j * lda]));
      den = fmax(den, fabs(a[i + (size_t)j * lda]));
    }
  return num / den;
}

int main(int argc, char **argv) {
  const int gpus = argc > 1 ? atoi(argv[1]) : 0;
  dplasma_context_t *ctx = dplasma_init(1, gpus);
  if (!ctx) return fail("init");
  int ok = 1;
  const int N = 160, NB = 32;
  double *a0 = malloc(sizeof(double) * N * N), *a = malloc(sizeof(double) * N * N);
  spd(a0, N, N);
  /* --- taskpool API on caller memory (CPU context: host memory in place) */
  if (gpus == 0) {
    memcpy(a, a0, sizeof(double) * N * N);
    dplasma_desc_t *A = dplasma_desc_block_cyclic_lapack(ctx, dplasmaRealDouble, NB, NB, N, N, 1, 1, 0, 0, a, N, 0);
    if (!A) return fail("desc_lapack");
    dplasma_taskpool_t *tp = dplasma_dpotrf_New(ctx, dplasmaLower, A);
    if (!tp) return fail("dpotrf_New");
    if (dplasma_context_add_taskpool(ctx, tp) != 0) return fail("add_taskpool");
    if (dplasma_context_start(ctx) != 0 || dplasma_context_wait(ctx) != 0) return fail("start/wait");
    const int info = dplasma_taskpool_result(tp);
    dplasma_dpotrf_Destruct(tp);
    dplasma_desc_destroy(A);
    const double r = chol_res(a, a0, N, N);
    printf("dpotrf_New info=%d res=%.3e\n", info, r);
    ok &= info == 0 && r < 1e-13;
  }
  /* --- ScaLAPACK layer on a 1 x 1 BLACS grid */
  parsec_init_wrapper_();
  int me, np, zero = 0, one = 1, ictxt, nprow, npcol, myrow, mycol, info;
  blacs_pinfo_(&me, &np);
  blacs_get_(&zero, &zero, &ictxt);
  blacs_gridinit_(&ictxt, "R", &one, &one);
  blacs_gridinfo_(&ictxt, &nprow, &npcol, &myrow, &mycol);
  int n = N, nb = NB, mloc = numroc_(&n, &nb, &myrow, &zero, &nprow), desca[9];
  descinit_(desca, &n, &n, &nb, &nb, &zero, &zero, &ictxt, &mloc, &info);
  memcpy(a, a0, sizeof(double) * N * N);
  pdpotrf_("L", &n, a, &one, &one, desca, &info);
  const double r2 = chol_res(a, a0, N, N);
  printf("pdpotrf_ info=%d res=%.3e grid=%dx%d\n", info, r2, nprow, npcol);
  ok &= info == 0 && r2 < 1e-13;
  /* pdtrsm_: X L^T = B with the factor above, checked by multiplying back */
  const int M = 50;
  int m = M, mloc2 = numroc_(&m, &nb, &myrow, &zero, &nprow), descb[9];
  descinit_(descb, &m, &n, &nb, &nb, &zero, &zero, &ictxt, &mloc2, &info);
  double *b = malloc(sizeof(double) * M * N), *b0 = malloc(sizeof(double) * M * N);
  for (int i = 0; i < M * N; ++i) b0[i] = b[i] = cos(0.1 * i);
  double alpha = 1.0;
  pdtrsm_("R", "L", "T", "N", &m, &n, &alpha, a, &one, &one, desca, b, &one, &one, descb);
  double e = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) {  /* (X L^T)(i, j) = sum_{k <= j} X(i, k) L(j, k) */
      double s = 0;
      for (int k = 0; k <= j; ++k) s += b[i + (size_t)k * M] * a[j + (size_t)k * N];
      e = fmax(e, fabs(s - b0[i + (size_t)j * M]));
    }
  printf("pdtrsm_ err=%.3e\n", e);
  ok &= e < 1e-12;
  /* pdgemm_: C = 0.5 A0 B^T + 2 C */
  double *c = malloc(sizeof(double) * M * N), *c0 = malloc(sizeof(double) * M * N);
  for (int i = 0; i < M * N; ++i) c0[i] = c[i] = sin(0.3 * i);
  double al = 0.5, be = 2.0;
  pdgemm_("N", "T", &m, &n, &n, &al, b0, &one, &one, descb, a0, &one, &one, desca, &be, c, &one, &one, descb);
  e = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += b0[i + (size_t)k * M] * a0[j + (size_t)k * N];
      e = fmax(e, fabs(0.5 * s + 2.0 * c0[i + (size_t)j * M] - c[i + (size_t)j * M]));
    }
  printf("pdgemm_ err=%.3e\n", e);
  ok &= e < 1e-11;
  /* pdgetrf_: PA = LU, checked through the pivots */
  int *ipiv = malloc(sizeof(int) * (mloc + NB));
  memcpy(a, a0, sizeof(double) * N * N);
  pdgetrf_(&n, &n, a, &one, &one, desca, ipiv, &info);
  double *pa = malloc(sizeof(double) * N * N);
  memcpy(pa, a0, sizeof(double) * N * N);
  for (int i = 0; i < N; ++i) {
    const int p = ipiv[i] - 1;
    if (p != i)
      for (int j = 0; j < N; ++j) {
        const double t = pa[i + (size_t)j * N];
        pa[i + (size_t)j * N] = pa[p + (size_t)j * N];
        pa[p + (size_t)j * N] = t;
      }
  }
  e = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double s = 0;
      for (int k = 0; k <= (i < j ? i : j); ++k) s += (k == i ? 1.0 : a[i + (size_t)k * N]) * a[k + (size_t)j * N];
      e = fmax(e, fabs(s - pa[i + (size_t)j * N]));
    }
  printf("pdgetrf_ info=%d err=%.3e\n", info, e);
  ok &= info == 0 && e < 1e-11;
  /* pdlatsqr_: workspace query (LWORK = -1) then the factorisation; the query must not touch A */
  {
    double *q = malloc(sizeof(double) * N * N), *tau = malloc(sizeof(double) * N), w1 = -1.0;
    int mq = N, nq = N, lwork = -1;
    memcpy(q, a0, sizeof(double) * N * N);
    pdlatsqr_(&mq, &nq, q, &one, &one, desca, tau, &w1, &lwork, &info);
    const double want = (double)NB * (N + N + NB);
    int same = memcmp(q, a0, sizeof(double) * N * N) == 0;
    printf("pdlatsqr_ query info=%d work(1)=%.0f (want %.0f) A untouched=%d\n", info, w1, want, same);
    ok &= info == 0 && w1 == want && same;
    lwork = (int)w1;
    double *work = malloc(sizeof(double) * lwork);
    pdlatsqr_(&mq, &nq, q, &one, &one, desca, tau, work, &lwork, &info);
    /* R^T R = A0^T A0 (R: upper triangle of the result) */
    double e = 0, d = 0;
    for (int j = 0; j < N; ++j)
      for (int i = 0; i <= j; ++i) {
        double s = 0, t = 0;
        for (int k = 0; k <= i; ++k) s += q[k + (size_t)i * N] * q[k + (size_t)j * N];
        for (int k = 0; k < N; ++k) t += a0[k + (size_t)i * N] * a0[k + (size_t)j * N];
        e = fmax(e, fabs(s - t));
        d = fmax(d, fabs(t));
      }
    printf("pdlatsqr_ info=%d |R'R - A'A|/|A'A| %.3e\n", info, e / d);
    ok &= info == 0 && e / d < 1e-12;
    free(q), free(tau), free(work);
  }
  blacs_gridexit_(&ictxt);
  parsec_fini_wrapper_();
  printf("%s\n", ok ? "SCALAPACK OK" : "SCALAPACK FAIL");
  return ok ? 0 : 2;
}
