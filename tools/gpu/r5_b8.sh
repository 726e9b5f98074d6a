#!/bin/bash
# r5 batch 8: row-pipelined high list (DPLASMA_DTR_LO_ORDER=rowpipe) -- 1-GPU DTR and the 2x4 emulation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b8
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
step tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_potrf_dtr.py || exit 1
DPLASMA_DTR_LO_ORDER=rowpipe step perf_rowpipe 400 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" || exit 1
step em16_2x4 200 python tools/emulate_potrf.py -N 16384 --grid 2x4 --order rowpipe --reps 1 --check --trace $O/em16_2x4.npz || exit 1
python tools/emul_trace.py $O/em16_2x4.npz 2 4 30 > $O/em16_2x4_chain.txt 2>&1
step em32_2x4 300 python tools/emulate_potrf.py -N 32768 --grid 2x4 --order rowpipe --reps 1 --trace $O/em32_2x4.npz || exit 1
python tools/emul_trace.py $O/em32_2x4.npz 2 4 64 > $O/em32_2x4_chain.txt 2>&1
step em64_2x4 400 python tools/emulate_potrf.py -N 65536 --grid 2x4 --order rowpipe --reps 1 || exit 1
rm -f $O/*.npz
exit 0
