#!/bin/bash
# r6 batch 30: new one-process DGETRF defaults (deferred left interchanges, look-ahead, 32-column pivoting blocks):
# LU GPU tests, then 32k / 64k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b30
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_lu.py tests/test_lu_qr.py tests/test_diag_cus_gpu.py tests/test_api_variants.py tests/test_capped.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for N in 16384 32768 65536; do
  for r in 1 2; do
    timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${N}_$r.log 2>&1 || { tail -5 $O/${N}_$r.log; exit 1; }
    grep TIME $O/${N}_$r.log | tail -1 | cut -c1-140 | tee -a $O/summary.log
  done
done
exit 0
