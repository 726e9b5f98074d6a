#!/bin/bash
# r4 batch 13: DTR gaps at 64k (trace analysis on the box, no file kept) and deeper deferral (longer tasks,
# fewer claims); then the round-end checks (full GPU suite, smoke, driver bench).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b13
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|gaps|next task|busy %" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_trace64k 240 python tools/gpu/dtr_trace_run.py 65536 || exit 1
for D in 6 8; do
  step dtr_D$D 300 env DPLASMA_DTR_DEFER=$D python tools/gpu/dtr_bench.py 65536 || exit 1
done
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python bench.py --steps 20 --warmup 5 || exit 1
grep -E '^\{' $O/bench.log | cut -c1-300
exit 0
