#!/bin/bash
# r4 batch 11: DTR tail (single-panel blocks once fewer than T columns remain) at 32k / 64k; LU rank replay
# (pivots of unmoved broadcasts clamped into the panel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b11
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|worst|pct_peak|rank [0-9]" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_trace64k 240 python tools/gpu/dtr_trace_run.py 65536 || exit 1
for T in 16 32; do
  step dtr_tail$T 400 env DPLASMA_DTR_DEFER_MIN_TILES=$T python tools/gpu/dtr_bench.py 32768 65536 || exit 1
done
step replay_python_2x4_bw65 500 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 2 --bw 65 --lat 10 || exit 1
step replay_python_2x4_bw65_noproxy 500 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --steps 2 --bw 65 --lat 10 --no-proxy || exit 1
step replay_native_2x4_bw65 400 python tools/replay_native.py -N 65536 --nb 512 --grid 2x4 --steps 2 --bw 65 --lat 10 || exit 1
exit 0
