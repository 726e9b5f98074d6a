#!/bin/bash
# Headline DPOTRF 64k on one GPU: register-resident panel TRSM (default) vs the batched engine, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
OUT=gpurun_out/b17_trsm_kind.log
: > $OUT
for rep in 1 2; do for K in rb gemm; do
  v=$(DPLASMA_POTRF_TRSM=$K timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-check 2>/dev/null | grep metric \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1000,2))") || exit 1
  echo "rep $rep TRSM=$K: $v TF/s" | tee -a $OUT
done; done
