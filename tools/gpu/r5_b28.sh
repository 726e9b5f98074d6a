#!/bin/bash
# r5 batch 28: native pltmg vs Python; native C suite; DTR 16k trace with one workgroup per CU (critical path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b28
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== capi native tests" | tee -a $O/summary.log
timeout -k 10 600 python -u -m pytest tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "native_gpu or native_pltmg" > $O/capi.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -3 $O/capi.log | tee -a $O/summary.log
echo "== dtr 16k trace (256 WGs)" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_trace_run.py 16384 $O/trace16k_256.npz > $O/trace16k.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
head -12 $O/trace16k.log | tee -a $O/summary.log
timeout -k 10 300 python tools/emul_critical.py $O/trace16k_256.npz 1 70 > $O/crit16k.log 2>&1
head -60 $O/crit16k.log | tee -a $O/summary.log
exit 0
