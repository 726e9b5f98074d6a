/* ScaLAPACK F77 layer without Python (one process, a GPU, 1 x 1 BLACS grid -> capi/native.cpp):
 * pdpotrf_, pdgemm_, pdgetrf_, pdtrsm_, pdtrmm_ on host local arrays, on submatrices (IA, JA > 1),
 * checked on the host; the embedded interpreter must never start. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dplasma.h"

static int fails = 0;
#define CHECK(c, ...)                                \
  do {                                               \
    if (!(c)) {                                      \
      printf("FAIL %s:%d ", __FILE__, __LINE__);     \
      printf(__VA_ARGS__);                           \
      printf("\n");                                  \
      fails++;                                       \
    }                                                \
  } while (0)

static void fill(double *x, size_t n, unsigned s) {
  for (size_t i = 0; i < n; ++i) {
    s = s * 1103515245u + 12345u;
    x[i] = ((s >> 8) & 0xffff) / 65536.0 - 0.5;
  }
}

int main(void) {
  setvbuf(stdout, NULL, _IONBF, 0);
  parsec_init_wrapper_();
  int me, np, zero = 0, one = 1, ictxt, nprow, npcol, myrow, mycol, info;
  blacs_pinfo_(&me, &np);
  blacs_get_(&zero, &zero, &ictxt);
  blacs_gridinit_(&ictxt, "R", &one, &one);
  blacs_gridinfo_(&ictxt, &nprow, &npcol, &myrow, &mycol);
  CHECK(np == 1 && nprow == 1 && npcol == 1 && myrow == 0 && mycol == 0, "grid %d %d %d %d", nprow, npcol, myrow, mycol);
  const int L = 220, N = 170, off = 21, nb = 64;   /* the N x N operand sits at (off, off) of an L x L array */
  int gl = L, nbv = nb, desca[9];
  descinit_(desca, &gl, &gl, &nbv, &nbv, &zero, &zero, &ictxt, &gl, &info);
  double *a = malloc(sizeof(double) * L * L), *a0 = malloc(sizeof(double) * L * L);
  fill(a0, (size_t)L * L, 3);
  /* SPD submatrix */
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += a0[(off - 1 + i) + (size_t)(off - 1 + k) * L] * a0[(off - 1 + j) + (size_t)(off - 1 + k) * L];
      a[(off - 1 + i) + (size_t)(off - 1 + j) * L] = s + (i == j ? N : 0.0);
    }
  for (int j = 0; j < L; ++j)
    for (int i = 0; i < L; ++i)
      if (i < off - 1 || j < off - 1 || i >= off - 1 + N || j >= off - 1 + N) a[i + (size_t)j * L] = a0[i + (size_t)j * L];
  double *spd = malloc(sizeof(double) * L * L);
  memcpy(spd, a, sizeof(double) * L * L);
  int n = N, ia = off;
  pdpotrf_("L", &n, a, &ia, &ia, desca, &info);
  double e = 0, d = 0;
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += a[(off - 1 + i) + (size_t)(off - 1 + k) * L] * a[(off - 1 + j) + (size_t)(off - 1 + k) * L];
      e = fmax(e, fabs(s - spd[(off - 1 + i) + (size_t)(off - 1 + j) * L]));
      d = fmax(d, fabs(spd[(off - 1 + i) + (size_t)(off - 1 + j) * L]));
    }
  int outside = 0;
  for (int j = 0; j < L; ++j)
    for (int i = 0; i < L; ++i)
      if ((i < off - 1 || j < off - 1 || i >= off - 1 + N || j >= off - 1 + N) && a[i + (size_t)j * L] != spd[i + (size_t)j * L]) outside++;
  printf("pdpotrf_ info=%d ||LL'-A||/||A|| %.3e (untouched outside: %d)\n", info, e / d, outside == 0);
  CHECK(info == 0 && e / d < 1e-13 && outside == 0, "pdpotrf_");

  /* pdgemm_: C(off..) = 0.5 A(off..) B^T + 2 C */
  double *b = malloc(sizeof(double) * L * L), *c = malloc(sizeof(double) * L * L), *c0 = malloc(sizeof(double) * L * L);
  fill(b, (size_t)L * L, 5), fill(c, (size_t)L * L, 6);
  memcpy(c0, c, sizeof(double) * L * L);
  double al = 0.5, be = 2.0;
  pdgemm_("N", "T", &n, &n, &n, &al, a0, &ia, &ia, desca, b, &ia, &ia, desca, &be, c, &ia, &ia, desca);
  e = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += a0[(off - 1 + i) + (size_t)(off - 1 + k) * L] * b[(off - 1 + j) + (size_t)(off - 1 + k) * L];
      e = fmax(e, fabs(0.5 * s + 2.0 * c0[(off - 1 + i) + (size_t)(off - 1 + j) * L] - c[(off - 1 + i) + (size_t)(off - 1 + j) * L]));
    }
  printf("pdgemm_ err=%.3e\n", e);
  CHECK(e < 1e-12, "pdgemm_ %.3e", e);

  /* pdgetrf_ on the general submatrix: P A = L U through the returned (global, 1-based) pivots */
  double *g = malloc(sizeof(double) * L * L);
  memcpy(g, a0, sizeof(double) * L * L);
  int *ipiv = malloc(sizeof(int) * (L + nb));
  pdgetrf_(&n, &n, g, &ia, &ia, desca, ipiv, &info);
  double *pa = malloc(sizeof(double) * N * N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) pa[i + (size_t)j * N] = a0[(off - 1 + i) + (size_t)(off - 1 + j) * L];
  int bad = 0;
  for (int i = 0; i < N; ++i) {
    const int p = ipiv[i] - off;   /* back to the submatrix's 0-based rows */
    if (p < i || p >= N) { bad++; continue; }
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
      for (int k = 0; k <= (i < j ? i : j); ++k) {
        const double l = k == i ? 1.0 : g[(off - 1 + i) + (size_t)(off - 1 + k) * L];
        s += l * g[(off - 1 + k) + (size_t)(off - 1 + j) * L];
      }
      e = fmax(e, fabs(s - pa[i + (size_t)j * N]));
    }
  printf("pdgetrf_ info=%d ||PA-LU|| %.3e bad pivots %d\n", info, e, bad);
  CHECK(info == 0 && e < 1e-12 && bad == 0, "pdgetrf_");

  /* pdtrsm_ then pdtrmm_ with the Cholesky factor: X = L^-1 B, then L X == B */
  memcpy(c0, b, sizeof(double) * L * L);
  double one_d = 1.0;
  pdtrsm_("L", "L", "N", "N", &n, &n, &one_d, a, &ia, &ia, desca, b, &ia, &ia, desca);
  pdtrmm_("L", "L", "N", "N", &n, &n, &one_d, a, &ia, &ia, desca, b, &ia, &ia, desca);
  e = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) e = fmax(e, fabs(b[(off - 1 + i) + (size_t)(off - 1 + j) * L] - c0[(off - 1 + i) + (size_t)(off - 1 + j) * L]));
  printf("pdtrsm_ + pdtrmm_ round trip err=%.3e\n", e);
  CHECK(e < 1e-10, "pdtrsm_/pdtrmm_ %.3e", e);

  blacs_gridexit_(&ictxt);
  parsec_fini_wrapper_();
  CHECK(dplasma_python_active() == 0, "the interpreter was started");
  printf("%s\n", fails ? "F77 NATIVE FAIL" : "F77 NATIVE OK");
  return fails ? 1 : 0;
}
