#!/bin/bash
# r6 batch 43: one-GPU DTR at 16k / 32k -- deferral depth D (DPLASMA_DTR_DEFER) with today's scheduler
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b43
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD DPLASMA_DTR_PLAN_CACHE=0
for d in 1 2 3 4 6; do
  DPLASMA_DTR_DEFER=$d timeout -k 10 300 python tools/gpu/dtr_bench.py --engine dtr --reps 4 16384 32768 > $O/d$d.log 2>&1 || { tail -5 $O/d$d.log; exit 1; }
  echo "D=$d $(grep -o 'N= [0-9]* .*gflops' $O/d$d.log | awk '{print $2, $(NF-1)}' | tr '\n' ' ')"
done
exit 0
