#!/bin/bash
# r6 batch 33: DTR priority weights A/B on one box (scan skip on): default (22 buckets, trsm 400 / potrf 800) vs
# 62 buckets with trsm 250 / potrf 500, three alternating rounds, 16k / 32k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b33
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for r in 1 2 3; do
  for cfg in "base:" "w:DPLASMA_DTR_BUCKETS=62 DPLASMA_DTR_BL_W=75,65,250,500"; do
    tag=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 300 python tools/gpu/dtr_bench.py --engine dtr --reps 4 16384 32768 > $O/${tag}_$r.log 2>&1 || { tail -5 $O/${tag}_$r.log; exit 1; }
    echo "$r $tag $(grep -o 'N= [0-9]* .*gflops' $O/${tag}_$r.log | awk '{print $2, $(NF-1)}' | tr '\n' ' ')" | tee -a $O/summary.log
  done
done
exit 0
