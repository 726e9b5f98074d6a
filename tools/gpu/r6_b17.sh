#!/bin/bash
# r6 batch 17: rocprofv3 PMC counters of the DTR Cholesky kernel at N = 16384 and 65536 (one pass per counter group)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r6b17
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
pass() {   # name N counters...
  local name=$1 n=$2; shift 2
  echo "== pass $name N=$n: $*" | tee -a $O/summary.log
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$name-$n -o p -- \
    python $R/tools/gpu/dtr_bench.py --engine dtr --reps 1 ${NOCHECK:-} $n > $O/$name-$n.log 2>&1 \
    || { tail -20 $O/$name-$n.log | tee -a $O/summary.log; return 1; }
  grep TIME $O/$name-$n.log | tee -a $O/summary.log
}
( while true; do date >> $O/heartbeat.log; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
for n in ${NS:-16384 65536}; do
  pass sq $n SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
  && pass l2 $n TCC_HIT_sum TCC_MISS_sum \
  && pass fetch $n FETCH_SIZE \
  && pass write $n WRITE_SIZE || exit 1
done
exit 0
