#!/bin/bash
# r5 batch 9: critical paths of the 1-GPU DTR (16k) and of the 2x4 emulation (16k, 32k; column order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b9
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|Error|error|TIME|EMUL|residual|span" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_potrf_dtr.py || exit 1
step tr1_16k 300 python tools/gpu/dtr_trace_run.py 16384 $O/g16.npz || exit 1
python tools/emul_critical.py $O/g16.npz 1 60 > $O/g16_critical.txt 2>&1
step em16_2x4 200 python tools/emulate_potrf.py -N 16384 --grid 2x4 --order column --reps 1 --check --trace $O/em16.npz || exit 1
python tools/emul_critical.py $O/em16.npz 8 80 > $O/em16_critical.txt 2>&1
step em32_2x4 300 python tools/emulate_potrf.py -N 32768 --grid 2x4 --order column --reps 1 --trace $O/em32.npz || exit 1
python tools/emul_critical.py $O/em32.npz 8 80 > $O/em32_critical.txt 2>&1
rm -f $O/*.npz
exit 0
