#!/bin/bash
# r5 batch 35: 2x4 push-scheduled grid emulation at 64k with the residual check; 4x2; 2x2 at 32k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b35
mkdir -p $O
export PYTHONUNBUFFERED=1
export DPLASMA_DTR_WG=256
em() {
  echo "== $1" | tee -a $O/summary.log
  shift
  DPLASMA_DTR_SCHED=queue timeout -k 10 400 python tools/emulate_potrf.py "$@" > $O/run.log 2>&1
  local rc=$?
  grep -E "EMUL|residual" $O/run.log | tail -2 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
em "2x4 64k check" -N 65536 --grid 2x4 --bw 50 --lat 10 --reps 2 --check || exit 1
em "2x4 64k bw 50 lat 15" -N 65536 --grid 2x4 --bw 50 --lat 15 --reps 2 || exit 1
em "4x2 64k" -N 65536 --grid 4x2 --bw 50 --lat 10 --reps 2 || exit 1
em "2x2 64k" -N 65536 --grid 2x2 --bw 50 --lat 10 --reps 2 || exit 1
em "1x2 64k" -N 65536 --grid 1x2 --bw 50 --lat 10 --reps 2 || exit 1
em "2x4 48k" -N 49152 --grid 2x4 --bw 50 --lat 10 --reps 2 || exit 1
exit 0
