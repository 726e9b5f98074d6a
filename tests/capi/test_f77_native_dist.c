/* ScaLAPACK F77 layer without Python on a P x Q BLACS grid of processes (RANK / WORLD_SIZE,
 * DPLASMA_NATIVE_RDV; capi/dplasma_f77.cpp -> the multi-process native engine): pdpotrf_, pdgemm_, pdtrsm_, pdgetrf_ on
 * each rank's ScaLAPACK local arrays (host memory), checked entry by entry against host arithmetic on the
 * global matrices (every rank holds the formulas); the embedded interpreter must never start.
 * usage (one process per rank): RANK=r WORLD_SIZE=w test_f77_native_dist nprow */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dplasma.h"

static int fails = 0, me = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      printf("FAIL rank %d %s:%d ", me, __FILE__, __LINE__); \
      printf(__VA_ARGS__);                              \
      printf("\n");                                     \
      fails++;                                          \
    }                                                   \
  } while (0)

static double fa(int i, int j) { return sin(0.37 * i + 1.3 * j) + 0.25 * cos(0.11 * i * j); }
static double fb(int i, int j) { return cos(0.23 * i - 0.7 * j); }
static double fc(int i, int j) { return 0.5 * sin(0.05 * (i + 3 * j)); }

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  const int nprow = argc > 1 ? atoi(argv[1]) : 1;
  int np, zero = 0, ictxt, P, Q, myrow, mycol, info;
  parsec_init_wrapper_();
  blacs_pinfo_(&me, &np);
  const int npcol = np / nprow;
  int pr = nprow, pc = npcol;
  blacs_get_(&zero, &zero, &ictxt);
  blacs_gridinit_(&ictxt, "R", &pr, &pc);
  blacs_gridinfo_(&ictxt, &P, &Q, &myrow, &mycol);
  CHECK(P == nprow && Q == npcol && myrow == me / npcol && mycol == me % npcol, "grid %d x %d at (%d, %d): %s", P, Q,
        myrow, mycol, dplasma_last_error());
  if (fails) return 1;
  const int N = 520, nb = 64;
  int n = N, nbv = nb, one = 1;
  const int lm = numroc_(&n, &nbv, &myrow, &zero, &P), ln = numroc_(&n, &nbv, &mycol, &zero, &Q);
  int lld = lm > 1 ? lm : 1, desc[9];
  descinit_(desc, &n, &n, &nbv, &nbv, &zero, &zero, &ictxt, &lld, &info);
  /* local (li, lj) <-> global (i, j) */
  int *gi = malloc(sizeof(int) * (lm + 1)), *gj = malloc(sizeof(int) * (ln + 1));
  for (int l = 0; l < lm; ++l) gi[l] = ((l / nb) * P + myrow) * nb + l % nb;
  for (int l = 0; l < ln; ++l) gj[l] = ((l / nb) * Q + mycol) * nb + l % nb;

  /* ---- pdpotrf_: SPD A = M M^T + N I (M = fa), lower */
  double *M = malloc(sizeof(double) * N * N), *S = malloc(sizeof(double) * N * N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) M[i + (size_t)j * N] = fa(i, j);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += M[i + (size_t)k * N] * M[j + (size_t)k * N];
      S[i + (size_t)j * N] = s + (i == j ? N : 0.0);
    }
  double *a = malloc(sizeof(double) * lld * (ln > 0 ? ln : 1));
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) a[li + (size_t)lj * lld] = S[gi[li] + (size_t)gj[lj] * N];
  pdpotrf_("L", &n, a, &one, &one, desc, &info);
  CHECK(info == 0, "pdpotrf_ info %d: %s", info, dplasma_last_error());
  double *S0 = malloc(sizeof(double) * N * N);
  memcpy(S0, S, sizeof(double) * N * N);
  /* host Cholesky of S (in place, lower) */
  for (int k = 0; k < N; ++k) {
    double d = sqrt(S[k + (size_t)k * N]);
    S[k + (size_t)k * N] = d;
    for (int i = k + 1; i < N; ++i) S[i + (size_t)k * N] /= d;
    for (int j = k + 1; j < N; ++j)
      for (int i = j; i < N; ++i) S[i + (size_t)j * N] -= S[i + (size_t)k * N] * S[j + (size_t)k * N];
  }
  double e = 0, nrm = 0;
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li)
      if (gi[li] >= gj[lj]) {
        const double y = S[gi[li] + (size_t)gj[lj] * N];
        e = fmax(e, fabs(a[li + (size_t)lj * lld] - y));
        nrm = fmax(nrm, fabs(y));
      }
  printf("rank %d: pdpotrf_ %dx%d grid, local max rel diff %.3e\n", me, P, Q, e / nrm);
  CHECK(e / nrm < 1e-12, "pdpotrf_ local entries differ by %.3e", e / nrm);

  /* ---- pdgemm_: C = 0.5 A B^T + 2 C */
  double *A = malloc(sizeof(double) * lld * (ln > 0 ? ln : 1)), *B = malloc(sizeof(double) * lld * (ln > 0 ? ln : 1));
  double *C = malloc(sizeof(double) * lld * (ln > 0 ? ln : 1));
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) {
      A[li + (size_t)lj * lld] = fa(gi[li], gj[lj]);
      B[li + (size_t)lj * lld] = fb(gi[li], gj[lj]);
      C[li + (size_t)lj * lld] = fc(gi[li], gj[lj]);
    }
  double al = 0.5, be = 2.0;
  pdgemm_("N", "T", &n, &n, &n, &al, A, &one, &one, desc, B, &one, &one, desc, &be, C, &one, &one, desc);
  e = 0, nrm = 0;
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) {
      double s = 0;
      for (int k = 0; k < N; ++k) s += fa(gi[li], k) * fb(gj[lj], k);
      const double y = al * s + be * fc(gi[li], gj[lj]);
      e = fmax(e, fabs(C[li + (size_t)lj * lld] - y));
      nrm = fmax(nrm, fabs(y));
    }
  printf("rank %d: pdgemm_ %dx%d grid, local max rel diff %.3e\n", me, P, Q, e / nrm);
  CHECK(e / nrm < 1e-12, "pdgemm_ local entries differ by %.3e", e / nrm);
  /* ---- pdtrsm_: X = 2 L^{-1} B0 with L the factor pdpotrf_ left in a (lower), B0 = fb */
  double *X = malloc(sizeof(double) * lld * (ln > 0 ? ln : 1));
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) X[li + (size_t)lj * lld] = fb(gi[li], gj[lj]);
  double two = 2.0;
  pdtrsm_("L", "L", "N", "N", &n, &n, &two, a, &one, &one, desc, X, &one, &one, desc);
  double *Xh = malloc(sizeof(double) * N * N);   /* host forward substitution on the global factor S */
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double v = 2.0 * fb(i, j);
      for (int k = 0; k < i; ++k) v -= S[i + (size_t)k * N] * Xh[k + (size_t)j * N];
      Xh[i + (size_t)j * N] = v / S[i + (size_t)i * N];
    }
  e = 0, nrm = 0;
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) {
      const double y = Xh[gi[li] + (size_t)gj[lj] * N];
      e = fmax(e, fabs(X[li + (size_t)lj * lld] - y));
      nrm = fmax(nrm, fabs(y));
    }
  printf("rank %d: pdtrsm_ %dx%d grid, local max rel diff %.3e\n", me, P, Q, e / nrm);
  CHECK(e / nrm < 1e-11, "pdtrsm_ local entries differ by %.3e", e / nrm);
  /* ---- pdgetrf_: LU with partial pivoting of fa on the grid against a host dgetf2 of the global matrix
   * (IPIV in ScaLAPACK layout: the global pivot row of each local row) */
  int *ipiv = malloc(sizeof(int) * (lm + nb));
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) A[li + (size_t)lj * lld] = fa(gi[li], gj[lj]);
  pdgetrf_(&n, &n, A, &one, &one, desc, ipiv, &info);
  CHECK(info == 0, "pdgetrf_ info %d: %s", info, dplasma_last_error());
  double *G = malloc(sizeof(double) * N * N);
  int *hp = malloc(sizeof(int) * N);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) G[i + (size_t)j * N] = fa(i, j);
  for (int k = 0; k < N; ++k) {
    int p = k;
    for (int i = k + 1; i < N; ++i)
      if (fabs(G[i + (size_t)k * N]) > fabs(G[p + (size_t)k * N])) p = i;
    hp[k] = p + 1;
    if (p != k)
      for (int j = 0; j < N; ++j) {
        const double t = G[k + (size_t)j * N];
        G[k + (size_t)j * N] = G[p + (size_t)j * N];
        G[p + (size_t)j * N] = t;
      }
    for (int i = k + 1; i < N; ++i) G[i + (size_t)k * N] /= G[k + (size_t)k * N];
    for (int j = k + 1; j < N; ++j)
      for (int i = k + 1; i < N; ++i) G[i + (size_t)j * N] -= G[i + (size_t)k * N] * G[k + (size_t)j * N];
  }
  int piv_ok = 1;
  for (int li = 0; li < lm; ++li) piv_ok = piv_ok && ipiv[li] == hp[gi[li]];
  e = 0, nrm = 0;
  for (int lj = 0; lj < ln; ++lj)
    for (int li = 0; li < lm; ++li) {
      const double y = G[gi[li] + (size_t)gj[lj] * N];
      e = fmax(e, fabs(A[li + (size_t)lj * lld] - y));
      nrm = fmax(nrm, fabs(y));
    }
  printf("rank %d: pdgetrf_ %dx%d grid, pivots %s, local max rel diff %.3e\n", me, P, Q, piv_ok ? "equal" : "DIFFER",
         e / nrm);
  CHECK(piv_ok && e / nrm < 1e-10, "pdgetrf_ pivots %d, local entries differ by %.3e", piv_ok, e / nrm);
  /* ---- unaligned operands (redistributed into an aligned copy and back, reference
   * scalapack_wrappers/common.c:27-128): the SPD matrix and a product at IA = JA = 38 of an (N + 37)^2
   * matrix distributed from process row P - 1; entries outside the operand must not change */
  {
    const int off = 37, N2 = N + off, rs = P - 1;
    int n2 = N2, rsv = rs, ia = off + 1;
    const int lm2 = numroc_(&n2, &nbv, &myrow, &rsv, &P), ln2 = numroc_(&n2, &nbv, &mycol, &zero, &Q);
    int lld2 = lm2 > 1 ? lm2 : 1, desc2[9];
    descinit_(desc2, &n2, &n2, &nbv, &nbv, &rsv, &zero, &ictxt, &lld2, &info);
    int *gi2 = malloc(sizeof(int) * (lm2 + 1)), *gj2 = malloc(sizeof(int) * (ln2 + 1));
    for (int l = 0; l < lm2; ++l) gi2[l] = ((l / nb) * P + (myrow - rs + P) % P) * nb + l % nb;
    for (int l = 0; l < ln2; ++l) gj2[l] = ((l / nb) * Q + mycol) * nb + l % nb;
    const size_t sz2 = (size_t)lld2 * (ln2 > 0 ? ln2 : 1);
    double *a2 = malloc(sizeof(double) * sz2), *c2 = malloc(sizeof(double) * sz2), *x2 = malloc(sizeof(double) * sz2);
    for (int lj = 0; lj < ln2; ++lj)
      for (int li = 0; li < lm2; ++li) {
        const int gI = gi2[li], gJ = gj2[lj];
        const int in = gI >= off && gJ >= off;
        a2[li + (size_t)lj * lld2] = in ? S0[(gI - off) + (size_t)(gJ - off) * N] : 100.0 + fa(gI, gJ);
        c2[li + (size_t)lj * lld2] = in ? fc(gI - off, gJ - off) : -100.0 - fb(gI, gJ);
        x2[li + (size_t)lj * lld2] = fa(gI, gJ);   /* the A operand of the product: rows/cols 38.. of x2 */
      }
    pdpotrf_("L", &n, a2, &ia, &ia, desc2, &info);
    CHECK(info == 0, "unaligned pdpotrf_ info %d: %s", info, dplasma_last_error());
    double e2 = 0, n2m = 0;
    int outside_ok = 1;
    for (int lj = 0; lj < ln2; ++lj)
      for (int li = 0; li < lm2; ++li) {
        const int gI = gi2[li], gJ = gj2[lj];
        const double v = a2[li + (size_t)lj * lld2];
        if (gI < off || gJ < off) {
          outside_ok = outside_ok && v == 100.0 + fa(gI, gJ);
        } else if (gI >= gJ) {
          const double y = S[(gI - off) + (size_t)(gJ - off) * N];
          e2 = fmax(e2, fabs(v - y));
          n2m = fmax(n2m, fabs(y));
        }
      }
    printf("rank %d: unaligned pdpotrf_ (IA=JA=%d, RSRC=%d) local max rel diff %.3e, outside %s\n", me, ia, rs,
           n2m > 0 ? e2 / n2m : 0.0, outside_ok ? "untouched" : "CHANGED");
    CHECK(outside_ok && (n2m == 0 || e2 / n2m < 1e-12), "unaligned pdpotrf_ diff %.3e", n2m > 0 ? e2 / n2m : 0.0);
    /* C(38.., 38..) = 0.5 X(38.., 38..) B^T + 2 C with B the aligned fb matrix of the first part */
    pdgemm_("N", "T", &n, &n, &n, &al, x2, &ia, &ia, desc2, B, &one, &one, desc, &be, c2, &ia, &ia, desc2);
    e2 = 0, n2m = 0, outside_ok = 1;
    for (int lj = 0; lj < ln2; ++lj)
      for (int li = 0; li < lm2; ++li) {
        const int gI = gi2[li], gJ = gj2[lj];
        const double v = c2[li + (size_t)lj * lld2];
        if (gI < off || gJ < off) {
          outside_ok = outside_ok && v == -100.0 - fb(gI, gJ);
          continue;
        }
        double sacc = 0;
        for (int k = 0; k < N; ++k) sacc += fa(gI, k + off) * fb(gJ - off, k);
        const double y = al * sacc + be * fc(gI - off, gJ - off);
        e2 = fmax(e2, fabs(v - y));
        n2m = fmax(n2m, fabs(y));
      }
    printf("rank %d: unaligned pdgemm_ local max rel diff %.3e, outside %s\n", me, n2m > 0 ? e2 / n2m : 0.0,
           outside_ok ? "untouched" : "CHANGED");
    CHECK(outside_ok && (n2m == 0 || e2 / n2m < 1e-12), "unaligned pdgemm_ diff %.3e", n2m > 0 ? e2 / n2m : 0.0);
    free(a2), free(c2), free(x2), free(gi2), free(gj2);
  }
  /* ---- pdlatsqr_: tall-skinny QR of fa (N x NS) on the grid; |R| = |chol(A^T A)^T| entry by entry (R's rows
   * are determined up to sign), tau in [1, 2] (real Householder) */
  {
    const int NS = 150;
    int ns = NS, lwork = -1;
    const int lnq = numroc_(&ns, &nbv, &mycol, &zero, &Q);
    int descq[9];
    descinit_(descq, &n, &ns, &nbv, &nbv, &zero, &zero, &ictxt, &lld, &info);
    double *q = malloc(sizeof(double) * lld * (lnq > 0 ? lnq : 1)), *tau = malloc(sizeof(double) * NS), wq = 0;
    for (int lj = 0; lj < lnq; ++lj)
      for (int li = 0; li < lm; ++li) q[li + (size_t)lj * lld] = fa(gi[li], gj[lj]);
    pdlatsqr_(&n, &ns, q, &one, &one, descq, tau, &wq, &lwork, &info);
    CHECK(info == 0 && wq > 0, "pdlatsqr_ workspace query: info %d work %g", info, wq);
    lwork = (int)wq;
    double *work = malloc(sizeof(double) * (lwork > 0 ? lwork : 1));
    pdlatsqr_(&n, &ns, q, &one, &one, descq, tau, work, &lwork, &info);
    CHECK(info == 0, "pdlatsqr_ info %d: %s", info, dplasma_last_error());
    double *G2 = malloc(sizeof(double) * NS * NS);   /* host Cholesky of A^T A (lower) */
    for (int j = 0; j < NS; ++j)
      for (int i = 0; i < NS; ++i) {
        double acc = 0;
        for (int k = 0; k < N; ++k) acc += fa(k, i) * fa(k, j);
        G2[i + (size_t)j * NS] = acc;
      }
    for (int k = 0; k < NS; ++k) {
      const double d = sqrt(G2[k + (size_t)k * NS]);
      G2[k + (size_t)k * NS] = d;
      for (int i = k + 1; i < NS; ++i) G2[i + (size_t)k * NS] /= d;
      for (int j = k + 1; j < NS; ++j)
        for (int i = j; i < NS; ++i) G2[i + (size_t)j * NS] -= G2[i + (size_t)k * NS] * G2[j + (size_t)k * NS];
    }
    double eq = 0, nq = 0;
    for (int lj = 0; lj < lnq; ++lj)
      for (int li = 0; li < lm; ++li)
        if (gi[li] <= gj[lj]) {   /* R(i, j) = +-L(j, i) */
          const double y = fabs(G2[gj[lj] + (size_t)gi[li] * NS]);
          eq = fmax(eq, fabs(fabs(q[li + (size_t)lj * lld]) - y));
          nq = fmax(nq, y);
        }
    int tau_ok = 1;
    for (int j = 0; j < NS; ++j) tau_ok = tau_ok && tau[j] >= 1.0 - 1e-12 && tau[j] <= 2.0 + 1e-12;
    printf("rank %d: pdlatsqr_ %dx%d on %dx%d grid: local max rel diff |R| %.3e, tau %s\n", me, N, NS, P, Q,
           nq > 0 ? eq / nq : 0.0, tau_ok ? "in [1, 2]" : "OUT OF RANGE");
    CHECK(tau_ok && (nq == 0 || eq / nq < 1e-11), "pdlatsqr_ |R| differs by %.3e", nq > 0 ? eq / nq : 0.0);
    free(q), free(tau), free(work), free(G2);
  }
  CHECK(!dplasma_python_active(), "the embedded interpreter was started");
  parsec_fini_wrapper_();
  if (fails) {
    printf("rank %d: F77 NATIVE DIST: %d FAILED\n", me, fails);
    return 1;
  }
  printf("rank %d: F77 NATIVE DIST OK\n", me);
  return 0;
}
