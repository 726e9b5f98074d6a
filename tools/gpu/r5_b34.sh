#!/bin/bash
# r5 batch 34: 2x4 grid emulation of the distributed DTR -- push scheduling vs lists (one workgroup per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b34
mkdir -p $O
export PYTHONUNBUFFERED=1
export DPLASMA_DTR_WG=256
echo "== gpu emulation tests" | tee -a $O/summary.log
timeout -k 10 300 python -u -m pytest tests/test_potrf_dtr.py -m gpu -x -q --timeout 200 --timeout-method thread -k emulation > $O/tests.log 2>&1
rc=$?
echo "rc=$rc" | tee -a $O/summary.log
tail -3 $O/tests.log | tee -a $O/summary.log
[ $rc -eq 0 ] || exit 1
for N in 16384 32768 65536; do
  echo "== queue 2x4 $N" | tee -a $O/summary.log
  DPLASMA_DTR_SCHED=queue timeout -k 10 300 python tools/emulate_potrf.py -N $N --grid 2x4 --bw 50 --lat 10 --reps 2 --check > $O/q_$N.log 2>&1
  echo "rc=$?" | tee -a $O/summary.log
  grep -E "EMUL|residual" $O/q_$N.log | tail -2 | tee -a $O/summary.log
done
echo "== queue 2x4 65536 bw 65" | tee -a $O/summary.log
DPLASMA_DTR_SCHED=queue timeout -k 10 300 python tools/emulate_potrf.py -N 65536 --grid 2x4 --bw 65 --lat 10 --reps 2 > $O/q_64k_65.log 2>&1
grep -E "EMUL" $O/q_64k_65.log | tail -1 | tee -a $O/summary.log
echo "== lists(step) 2x4 32768 (256 WGs)" | tee -a $O/summary.log
DPLASMA_DTR_SCHED=lists timeout -k 10 300 python tools/emulate_potrf.py -N 32768 --grid 2x4 --bw 50 --lat 10 --reps 2 > $O/l_32k.log 2>&1
grep -E "EMUL" $O/l_32k.log | tail -1 | tee -a $O/summary.log
exit 0
