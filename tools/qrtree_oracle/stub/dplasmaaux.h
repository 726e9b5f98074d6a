#ifndef ORACLE_DPLASMAAUX_H
#define ORACLE_DPLASMAAUX_H
#include <stdio.h>
#define dplasma_error(f, m) do { fprintf(stderr, "%s: %s\n", f, m); } while (0)
#define dplasma_warning(f, m) do { fprintf(stderr, "%s: %s\n", f, m); } while (0)
#define dplasma_inform(...) do {} while (0)
#endif
