#!/bin/bash
# r5 batch 5: single-rank DTR after the operand-offset prefetch; emulation traces (16k 2x4 / 1x2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b5
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|Error|error|TIME|EMUL|residual" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step perf 300 python tools/gpu/dtr_bench.py 16384 32768 || exit 1
step em16_2x4 200 python tools/emulate_potrf.py -N 16384 --grid 2x4 --reps 1 --trace $O/em16_2x4.npz || exit 1
python tools/emul_trace.py $O/em16_2x4.npz 2 4 30 > $O/em16_2x4_chain.txt 2>&1
step em16_1x2 200 python tools/emulate_potrf.py -N 16384 --grid 1x2 --reps 1 --trace $O/em16_1x2.npz || exit 1
python tools/emul_trace.py $O/em16_1x2.npz 1 2 30 > $O/em16_1x2_chain.txt 2>&1
rm -f $O/*.npz
exit 0
