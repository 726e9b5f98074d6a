#!/bin/bash
# r5 batch 15: catch a failing traced run of the segmented step order (STEPW=8) and check it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b15
mkdir -p $O
export PYTHONUNBUFFERED=1
export DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8
DTR_TRACE_RUNS=24 timeout -k 10 500 python tools/gpu/dtr_trace_run.py 32768 $O/g32.npz > $O/tr32.log 2>&1
echo "rc=$?" >> $O/tr32.log
grep -E "check=False|span|rc=" $O/tr32.log; grep -c "check=True" $O/tr32.log
timeout 300 python tools/emul_critical.py $O/g32.npz 1 10 > $O/g32_check.txt 2>&1
head -16 $O/g32_check.txt
rm -f $O/*.npz
exit 0
