#!/bin/bash
# r4 batch 24: pivoting block kernel with one barrier per local / global pivot search (the waves' winners are
# reduced by every thread from LDS); then the round-end checks (full GPU suite, smoke, the driver's bench) and
# the HQR 2x4 rank replay.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b24
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|smoke|worst|rank .*ms|us/column" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step lu_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lu.py tests/test_lu_qr.py -m gpu || exit 1
step lu_block 120 python tools/gpu/lu_block_bench.py 8192 32768 65536 || exit 1
step getrf32k 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf64k 300 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 || exit 1
step luqr32k 300 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python bench.py --steps 20 --warmup 5 || exit 1
grep -E '^\{' $O/bench.log | cut -c1-300
step hqr_replay_2x4 900 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks all --bw 65 --lat 10 || exit 1
exit 0
