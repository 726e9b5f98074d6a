#!/bin/bash
# r5 batch 12: hunt the intermittent wrong factor of the segmented step order: traced 32k runs until one fails,
# then the dependency checker on that trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b12
mkdir -p $O
export PYTHONUNBUFFERED=1
export DPLASMA_DTR_LO_ORDER=step
DTR_TRACE_RUNS=6 timeout -k 10 400 python tools/gpu/dtr_trace_run.py 32768 $O/g32.npz > $O/tr32.log 2>&1
echo "rc=$?" >> $O/tr32.log
grep -E "run |span|rc=" $O/tr32.log
timeout 300 python tools/emul_critical.py $O/g32.npz 1 20 > $O/g32_check.txt 2>&1
head -20 $O/g32_check.txt
rm -f $O/*.npz
exit 0
