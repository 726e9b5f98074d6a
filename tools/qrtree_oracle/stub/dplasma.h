/* Minimal stand-ins for the declarations the reference's QR-tree source files use (tools/qrtree_oracle):
 * integer helpers, enums and a tiled-matrix header with the mt / nt fields the trees read. */
#ifndef ORACLE_DPLASMA_H
#define ORACLE_DPLASMA_H
#include <stdio.h>
#include <stdlib.h>
#include <assert.h>
#define BEGIN_C_DECLS
#define END_C_DECLS
typedef int dplasma_enum_t;
#define dplasmaNoTrans 111
#define dplasmaTrans 112
#define dplasmaConjTrans 113
typedef struct { int nodes; } parsec_data_collection_stub_t;
typedef struct parsec_tiled_matrix_s { parsec_data_collection_stub_t super; int mt, nt, mb, nb, m, n, lmt, lnt; } parsec_tiled_matrix_t;
static inline int dplasma_imax(int a, int b) { return a > b ? a : b; }
static inline int dplasma_imin(int a, int b) { return a < b ? a : b; }
static inline int dplasma_iceil(int a, int b) { return (a + b - 1) / b; }
#endif
