/* Reference oracle for the QR elimination trees: links the reference's OWN tree sources
 * (/root/reference/src/dplasma_hqr.c, dplasma_systolic_qr.c, compiled here from source by
 * tools/qrtree_oracle/build.sh) and prints, for each parameter set given on the command line, the
 * complete tree as JSON: per step k the geqrt list (getm) and per row m its type, currpiv, and the
 * nextpiv / prevpiv chains.  tests/test_qrtree_parity.py compares dplasma_amd.models.qrtree with the
 * stored output (tests/fixtures/qrtree_ref.json), so the parity is against the reference's code
 * itself, not a re-derivation.
 *   usage: oracle hqr  MT NT llvl hlvl a p domino tsrr
 *          oracle svd  MT NT hlvl p cores ratio
 *          oracle sys  MT NT p q */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dplasma.h"
#include "dplasma/qr_param.h"

static void dump(const dplasma_qrtree_t *t, int mt, int nt) {
  const int kt = mt < nt ? mt : nt;
  printf("{\"mt\": %d, \"nt\": %d, \"steps\": [", mt, nt);
  for (int k = 0; k < kt; ++k) {
    printf("%s{\"k\": %d, \"getm\": [", k ? ", " : "", k);
    const int ng = t->getnbgeqrf(t, k);
    for (int i = 0; i < ng; ++i) printf("%s%d", i ? ", " : "", t->getm(t, k, i));
    printf("], \"rows\": [");
    for (int m = k; m < mt; ++m) {
      printf("%s[%d, %d, %d, [", m > k ? ", " : "", m, t->gettype(t, k, m), m > k ? t->currpiv(t, k, m) : -1);
      /* nextpiv chain of m as an annihilator, from "start" (mt) */
      int first = 1, guard = 0;
      for (int n = t->nextpiv(t, k, m, mt); n != mt && guard < 4 * mt; n = t->nextpiv(t, k, m, n), ++guard) {
        printf("%s%d", first ? "" : ", ", n);
        first = 0;
      }
      printf("], [");
      first = 1, guard = 0;
      for (int n = t->prevpiv(t, k, m, m); n != mt && guard < 4 * mt; n = t->prevpiv(t, k, m, n), ++guard) {
        printf("%s%d", first ? "" : ", ", n);
        first = 0;
      }
      printf("]]");
    }
    printf("]}");
  }
  printf("]}\n");
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  dplasma_qrtree_t t;
  parsec_tiled_matrix_t A;
  memset(&A, 0, sizeof A);
  if (!strcmp(argv[1], "hqr") && argc == 10) {
    A.mt = atoi(argv[2]), A.nt = atoi(argv[3]);
    if (dplasma_hqr_init(&t, dplasmaNoTrans, &A, atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]),
                         atoi(argv[8]), atoi(argv[9])) != 0) return 3;
    dump(&t, A.mt, A.nt);
    dplasma_hqr_finalize(&t);
    return 0;
  }
  if (!strcmp(argv[1], "svd") && argc == 8) {
    A.mt = atoi(argv[2]), A.nt = atoi(argv[3]);
    A.super.nodes = atoi(argv[5]);   /* one node per distributed-tree member */
    if (dplasma_svd_init(&t, dplasmaNoTrans, &A, atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7])) != 0)
      return 3;
    dump(&t, A.mt, A.nt);
    dplasma_hqr_finalize(&t);
    return 0;
  }
  if (!strcmp(argv[1], "sys") && argc == 6) {
    A.mt = atoi(argv[2]), A.nt = atoi(argv[3]);
    if (dplasma_systolic_init(&t, dplasmaNoTrans, &A, atoi(argv[4]), atoi(argv[5])) != 0) return 3;
    dump(&t, A.mt, A.nt);
    dplasma_systolic_finalize(&t);
    return 0;
  }
  return 2;
}
