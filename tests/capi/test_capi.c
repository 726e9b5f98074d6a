/* C-ABI smoke test: the reference's testing_dpotrf / testing_dgemm flow from plain C.
 * usage: test_capi <gpus> <N> <NB>   (gpus = 0: CPU reference path) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "dplasma.h"

static int fail(const char *what) {
  fprintf(stderr, "FAIL %s: %s\n", what, dplasma_last_error());
  return 1;
}

int main(int argc, char **argv) {
  const int gpus = argc > 1 ? atoi(argv[1]) : 0;
  const int N = argc > 2 ? atoi(argv[2]) : 300, NB = argc > 3 ? atoi(argv[3]) : 64;
  dplasma_context_t *ctx = dplasma_init(1, gpus);
  if (!ctx) return fail("init");
  /* --- Cholesky of dplghe(bump=N, seed 3872), residual ||L L^T - A|| / ||A|| computed in C */
  dplasma_desc_t *A = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, N, 1, 1, dplasmaUpperLower);
  if (!A) return fail("desc");
  if (dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, A, 3872ULL) != 0) return fail("plghe");
  double *a0 = malloc(sizeof(double) * N * N), *l = malloc(sizeof(double) * N * N);
  if (dplasma_desc_get_lapack(A, a0, N) != 0) return fail("get");
  int info = dplasma_dpotrf(ctx, dplasmaLower, A);
  if (info != 0) return fail("potrf");
  dplasma_desc_get_lapack(A, l, N);
  double num = 0, den = 0;
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += l[i + (size_t)k * N] * l[j + (size_t)k * N];
      num = fmax(num, fabs(s - a0[i + (size_t)j * N]));
      den = fmax(den, fabs(a0[i + (size_t)j * N]));
    }
  const double rel = num / den;
  printf("dpotrf N=%d NB=%d info=%d rel=%.3e\n", N, NB, info, rel);
  /* --- GEMM with host-provided operands, checked against a C triple loop */
  const int M = 70, K = 45, P = 53;
  double *ha = malloc(sizeof(double) * M * K), *hb = malloc(sizeof(double) * K * P), *hc = malloc(sizeof(double) * M * P);
  for (int i = 0; i < M * K; ++i) ha[i] = sin(i);
  for (int i = 0; i < K * P; ++i) hb[i] = cos(i);
  for (int i = 0; i < M * P; ++i) hc[i] = 0.5 * i / (M * P);
  dplasma_desc_t *dA = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, 16, 16, M, K, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *dB = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, 16, 16, K, P, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *dC = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, 16, 16, M, P, 0, 0, dplasmaUpperLower);
  dplasma_desc_set_lapack(dA, ha, M);
  dplasma_desc_set_lapack(dB, hb, K);
  dplasma_desc_set_lapack(dC, hc, M);
  if (dplasma_dgemm(ctx, dplasmaNoTrans, dplasmaNoTrans, 0.51, dA, dB, -0.42, dC) != 0) return fail("gemm");
  double *out = malloc(sizeof(double) * M * P), err = 0;
  dplasma_desc_get_lapack(dC, out, M);
  for (int j = 0; j < P; ++j)
    for (int i = 0; i < M; ++i) {
      double s = 0;
      for (int k = 0; k < K; ++k) s += ha[i + k * M] * hb[k + j * K];
      err = fmax(err, fabs(out[i + j * M] - (0.51 * s - 0.42 * hc[i + j * M])));
    }
  const double nrm = dplasma_dlange(ctx, dplasmaMaxNorm, dC);
  printf("dgemm err=%.3e lange(max)=%.6f\n", err, nrm);
  /* --- a complex entry point: zplrnt + zlange */
  dplasma_desc_t *Z = dplasma_desc_block_cyclic(ctx, dplasmaComplexDouble, 16, 16, 40, 40, 0, 0, dplasmaUpperLower);
  dplasma_zplrnt(ctx, 0, Z, 77ULL);
  const double zn = dplasma_zlange(ctx, dplasmaFrobeniusNorm, Z);
  printf("zlange(fro)=%.6f\n", zn);
  dplasma_desc_destroy(Z);
  dplasma_desc_destroy(dA);
  dplasma_desc_destroy(dB);
  dplasma_desc_destroy(dC);
  dplasma_desc_destroy(A);
  dplasma_fini(ctx);
  const int ok = rel < 1e-12 && err < 1e-12 && zn > 0 && isfinite(nrm);
  printf("%s\n", ok ? "CAPI OK" : "CAPI FAIL");
  return ok ? 0 : 2;
}
