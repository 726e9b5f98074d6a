#!/bin/bash
# Interpreter-free C ABI on the GPU: the native test program (checks + dpotrf timings at 32k / 64k)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
gcc -O2 -g -o gpurun_out/test_native tests/capi/test_native.c -Icapi/include -Ldplasma_amd/lib -ldplasma -lm \
    -Wl,-rpath,$R/dplasma_amd/lib || exit 1
for N in ${NATIVE_N:-0 32768 65536}; do
  timeout -k 10 300 ./gpurun_out/test_native $N > gpurun_out/native_$N.log 2>&1
  rc=$?
  tail -45 gpurun_out/native_$N.log
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; }
done
