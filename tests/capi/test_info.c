/* dplasma_info_t through the C ABI: set / replace / delete / enumerate / get (the behaviour the
 * reference checks in tests/testing_info.c).  Returns the number of failed checks. */
#include <stdio.h>
#include <string.h>

#include "dplasma.h"

static int check(int cond, const char *what) {
  if (!cond) fprintf(stderr, "info check failed: %s\n", what);
  return cond ? 0 : 1;
}

int main(void) {
  dplasma_info_t info;
  char key[DPLASMA_MAX_INFO_KEY + 1], value[DPLASMA_MAX_INFO_VAL];
  int n = 0, present = 0, errors = 0, seen_b = 0, seen_c = 0;
  dplasma_info_create(&info);
  dplasma_info_set(info, "KEYA", "VALUEA");
  dplasma_info_set(info, "KEYB", "VALUEB1");
  dplasma_info_set(info, "KEYC", "VALUEC");
  dplasma_info_set(info, "KEYB", "VALUEB2");   /* replaces */
  errors += check(dplasma_info_delete(info, "KEYA") == 0, "delete existing");
  errors += check(dplasma_info_delete(info, "NONKEY") != 0, "delete missing reports");
  dplasma_info_get_nkeys(info, &n);
  errors += check(n == 2, "two keys left");
  for (int i = 0; i < n; ++i) {
    dplasma_info_get_nthkey(info, i, key);
    if (!strcmp(key, "KEYB")) seen_b++;
    else if (!strcmp(key, "KEYC")) seen_c++;
    else errors += check(0, "unexpected key");
  }
  errors += check(seen_b == 1 && seen_c == 1, "each key enumerated once");
  dplasma_info_get(info, "KEYA", sizeof value, value, &present);
  errors += check(!present, "deleted key absent");
  dplasma_info_get(info, "KEYB", sizeof value, value, &present);
  errors += check(present && !strcmp(value, "VALUEB2"), "replaced value");
  dplasma_info_get(info, "KEYC", sizeof value, value, &present);
  errors += check(present && !strcmp(value, "VALUEC"), "kept value");
  errors += check(dplasma_info_get_nthkey(info, 5, key) != 0, "nthkey out of range");
  dplasma_info_free(&info);
  errors += check(info == NULL, "free clears the handle");
  printf("%s (%d errors)\n", errors ? "INFO FAIL" : "INFO OK", errors);
  return errors;
}
