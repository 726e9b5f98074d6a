#!/bin/bash
# Upper DPOTRF via the transposed lower schedule: GPU kernel tests, then lower vs upper 16k/32k/64k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/r3_upper.log; : > $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "potrf or swap" --timeout 150 \
    --timeout-method thread > gpurun_out/r3_upper_tests.log 2>&1 || { tail -30 gpurun_out/r3_upper_tests.log; exit 1; }
tail -2 gpurun_out/r3_upper_tests.log >> $out
for N in 16384 32768 65536; do for U in L U; do
  timeout -k 10 300 python bench.py -N $N --uplo $U --steps 3 --warmup 1 2>&1 | grep -E "TIME|\"check\"" | cut -c1-150 >> $out || { tail -20 $out; exit 1; }
done; done
DPLASMA_POTRF_UPPER=native timeout -k 10 200 python bench.py -N 16384 --uplo U --steps 3 --warmup 1 2>&1 | grep TIME >> $out
grep -v amdgpu.ids $out
