/* Out-of-tree example (reference: examples/ + the installed dplasma.h): Cholesky factorisation and
 * solve of a random SPD system through the installed C library.
 *   cmake -S examples -B build -DCMAKE_PREFIX_PATH=<prefix> && cmake --build build && build/potrf_example 0
 *   cc examples/potrf_example.c $(pkg-config --cflags --libs dplasma) -lm -o potrf_example
 * argument: number of GPUs (0 = CPU reference path) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "dplasma.h"

int main(int argc, char **argv) {
  const int gpus = argc > 1 ? atoi(argv[1]) : 0;
  const int N = 400, NB = 64, NRHS = 3;
  dplasma_context_t *ctx = dplasma_init(1, gpus);
  if (!ctx) { fprintf(stderr, "init: %s\n", dplasma_last_error()); return 1; }
  dplasma_desc_t *A = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, N, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *B = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, NRHS, 0, 0, dplasmaUpperLower);
  dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, A, 51ULL);
  dplasma_dplrnt(ctx, 0, B, 52ULL);
  double *a = malloc(sizeof(double) * N * N), *b = malloc(sizeof(double) * N * NRHS),
         *x = malloc(sizeof(double) * N * NRHS);
  dplasma_desc_get_lapack(A, a, N);
  dplasma_desc_get_lapack(B, b, N);
  /* non-blocking flavour: build the taskpool, run it, read its info */
  dplasma_taskpool_t *tp = dplasma_dpotrf_New(ctx, dplasmaLower, A);
  dplasma_context_add_taskpool(ctx, tp);
  dplasma_context_start(ctx);
  dplasma_context_wait(ctx);
  const int info = dplasma_taskpool_result(tp);
  dplasma_dpotrf_Destruct(tp);
  if (info != 0 || dplasma_dpotrs(ctx, dplasmaLower, A, B) != 0) { fprintf(stderr, "potrf/potrs failed\n"); return 1; }
  dplasma_desc_get_lapack(B, x, N);
  double r = 0, nb = 0;
  for (int c = 0; c < NRHS; ++c)
    for (int i = 0; i < N; ++i) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += a[(i >= k) ? i + (size_t)k * N : k + (size_t)i * N] * x[k + (size_t)c * N];
      r = fmax(r, fabs(s - b[i + (size_t)c * N]));
      nb = fmax(nb, fabs(b[i + (size_t)c * N]));
    }
  printf("potrf_example N=%d info=%d ||Ax-b||/||b|| = %.3e %s\n", N, info, r / nb, r / nb < 1e-10 ? "OK" : "FAIL");
  dplasma_desc_destroy(A);
  dplasma_desc_destroy(B);
  dplasma_fini(ctx);
  return r / nb < 1e-10 ? 0 : 2;
}
