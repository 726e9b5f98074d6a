/* Interpreter-free multi-process example: one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK, as set by
 * torchrun or mpirun wrappers), a P x Q grid, a distributed Cholesky solve checked through the norms, then a
 * timed DPOTRF in the reference tester's [****] format (tests/common.h:269-276).
 *   DPLASMA_NATIVE_RDV=/tmp/rdv.$$ torchrun --nproc-per-node 8 --no-python native_dist_example 65536 512 2
 * arguments: N (default 4096), NB (512), P (process rows, default 1) */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "dplasma.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 4096, NB = argc > 2 ? atoi(argv[2]) : 512, P = argc > 3 ? atoi(argv[3]) : 1;
  const char *r = getenv("RANK"), *w = getenv("WORLD_SIZE"), *lr = getenv("LOCAL_RANK");
  const int rank = r ? atoi(r) : 0, world = w ? atoi(w) : 1, dev = lr ? atoi(lr) : 0;
  dplasma_context_t *ctx = dplasma_init_native_dist(dev, rank, world, P, NULL);
  if (!ctx) { fprintf(stderr, "rank %d: init: %s\n", rank, dplasma_last_error()); return 1; }
  const int NRHS = 16;
  dplasma_desc_t *A = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, N, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *A0 = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, N, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *B = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, NRHS, 0, 0, dplasmaUpperLower);
  dplasma_desc_t *X = dplasma_desc_block_cyclic(ctx, dplasmaRealDouble, NB, NB, N, NRHS, 0, 0, dplasmaUpperLower);
  if (!A || !A0 || !B || !X) { fprintf(stderr, "rank %d: descriptors: %s\n", rank, dplasma_last_error()); return 1; }
  /* solve A X = B and check ||A X - B|| / (||A|| ||X|| N eps) with a distributed GEMM */
  dplasma_dplghe(ctx, (double)N, dplasmaLower, A, 3872);
  dplasma_dplghe(ctx, (double)N, dplasmaUpperLower, A0, 3872);
  dplasma_dplrnt(ctx, 0, B, 2354);
  dplasma_dlacpy(ctx, dplasmaUpperLower, B, X);
  const int info = dplasma_dposv(ctx, dplasmaLower, A, X);
  const double an = dplasma_dlange(ctx, dplasmaInfNorm, A0), xn = dplasma_dlange(ctx, dplasmaInfNorm, X);
  dplasma_dgemm(ctx, dplasmaNoTrans, dplasmaNoTrans, 1.0, A0, X, -1.0, B);
  const double res = dplasma_dlange(ctx, dplasmaInfNorm, B) / (an * xn * N * 1.1102230246251565e-16);
  if (rank == 0) printf("dposv N=%d NB=%d grid %dx%d: info %d, scaled residual %.3e (%s)\n", N, NB, P, world / P, info,
                        res, info == 0 && res < 60.0 ? "ok" : "FAILED");
  /* timed factorisation: taskpool built outside the timed region, ranks aligned by a norm (an all-reduce) */
  dplasma_dplghe(ctx, (double)N, dplasmaLower, A, 3872);
  dplasma_taskpool_t *tp = dplasma_dpotrf_New(ctx, dplasmaLower, A);
  (void)dplasma_dlange(ctx, dplasmaMaxNorm, B);
  const double t0 = now();
  dplasma_context_add_taskpool(ctx, tp);
  dplasma_context_start(ctx);
  dplasma_context_wait(ctx);
  (void)dplasma_dlange(ctx, dplasmaMaxNorm, B);
  const double t = now() - t0;
  const double fl = ((double)N * N * N / 3.0 + (double)N * N / 2.0 + N / 6.0) / 1e9;
  if (rank == 0)
    printf("[****] TIME(s) %12.5f : dpotrf PxQxg= %3d %-3d %d NB= %4d N= %7d : %14f gflops\n", t, P, world / P, 1, NB, N,
           fl / t);
  dplasma_dpotrf_Destruct(tp);
  dplasma_desc_destroy(A), dplasma_desc_destroy(A0), dplasma_desc_destroy(B), dplasma_desc_destroy(X);
  dplasma_fini(ctx);
  return info == 0 && res < 60.0 ? 0 : 1;
}
