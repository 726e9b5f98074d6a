#!/bin/bash
# Fused tile POTRF + panel TRSM: numerics (tile level, whole factorisation), then rb vs fused timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_potrf_tile_gpu.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/fused_tests.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/fused_tests.log | head; tail -5 gpurun_out/fused_tests.log; exit 1; }
tail -1 gpurun_out/fused_tests.log
for N in 16384 32768 65536; do
  for tk in rb fused; do
    st=3; [ $N -eq 65536 ] && st=2
    echo -n "N=$N TRSM=$tk " ; DPLASMA_POTRF_TRSM=$tk timeout -k 10 150 python bench.py -N $N --steps $st --warmup 1 \
        --no-check 2>&1 | grep TIME || exit 1
  done
done
DPLASMA_POTRF_TRSM=fused timeout -k 10 150 python bench.py -N 32768 --steps 1 --warmup 1 2>&1 | grep -E "SUCCESS|FAIL|TIME" || exit 1
