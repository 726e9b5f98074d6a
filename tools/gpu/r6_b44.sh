#!/bin/bash
# r6 batch 44: one-GPU DTR, one vs two workgroups per CU with the scan skip (alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b44
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for r in 1 2; do
  for w in 256 512; do
    DPLASMA_DTR_WG=$w timeout -k 10 300 python tools/gpu/dtr_bench.py --engine dtr --reps 3 16384 32768 65536 > $O/w${w}_$r.log 2>&1 || { tail -5 $O/w${w}_$r.log; exit 1; }
    echo "WG=$w $(grep -o 'N= [0-9]* .*check=[A-Za-z]*' $O/w${w}_$r.log | awk '{print $2, $(NF-2), $NF}' | tr '\n' ' ')"
  done
done
exit 0
