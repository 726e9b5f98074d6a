#!/bin/bash
# r6 batch 38: DTR 16k -- are the slow early POTRFs waiting on dirty lines of the NEAR updates? write-through update /
# TRSM stores (DPLASMA_DTR_WT=1) and system-scope acquire (DPLASMA_DTR_SYSACQ=1), traced
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b38
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "wt:DPLASMA_DTR_WT=1" "sysacq:DPLASMA_DTR_SYSACQ=1"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python -u tools/gpu/dtr_trace_run.py 16384 > $O/$tag.log 2>&1 || { tail -10 $O/$tag.log; exit 1; }
  echo "== $tag: $(grep '^N=' $O/$tag.log)"
  grep -A3 "^POTRF(1)" $O/$tag.log | grep "W end"
  grep -A3 "^POTRF(5)" $O/$tag.log | grep "W end"
done
exit 0
