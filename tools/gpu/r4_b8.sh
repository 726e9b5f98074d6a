#!/bin/bash
# r4 batch 8: native grid engine (QR, new Cholesky schedule, F77 redistribution + pdlatsqr_) C tests;
# rank replays: native vs Python Cholesky 2x4, LU (getrf_ptgpanel) 2x4 at xlat 16 / 6 us per column.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b8
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|FAIL|error|Error|worst|pct_peak|rank [0-9]" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step capi_native 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi.py -m gpu -k "native" || exit 1
step replay_native_2x4 400 python tools/replay_native.py -N 65536 --nb 512 --grid 2x4 --steps 1 || exit 1
step replay_python_2x4_noproxy 500 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 1 --no-proxy || exit 1
step replay_python_2x4 500 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 1 || exit 1
step replay_python_2x4_cap16 500 env DPLASMA_POTRF_BULK_CAP=16 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 1 || exit 1
step replay_python_2x4_cap32 500 env DPLASMA_POTRF_BULK_CAP=32 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 1 || exit 1
exit 0
