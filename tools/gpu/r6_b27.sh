#!/bin/bash
# r6 batch 27: 2x4 LU rehearsal (gather panels) -- repeatability, look-ahead off, RNF on, N variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b27
mkdir -p $O
export DPLASMA_DIST_BACKEND=gloo PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 \
    --master-port $((29650 + RANDOM % 200)) tools/gpu/lu_dist_rehearsal.py ${NN:-4096} 256 2 > $O/$tag.log 2>&1
  echo "== $tag rc=$?: $(grep -o 'max |factor diff| [0-9.e+-]* : [A-Z]*' $O/$tag.log | sort | uniq -c | tr '\n' ' ')"
}
run gather1 DPLASMA_LU_PANEL=gather
run gather2 DPLASMA_LU_PANEL=gather
run gather3 DPLASMA_LU_PANEL=gather
run gather_rnf DPLASMA_LU_PANEL=gather DPLASMA_LU_RNF=1
run gather_la0 DPLASMA_LU_PANEL=gather DPLASMA_LU_LOOKAHEAD=0
run gather_ch1 DPLASMA_LU_PANEL=gather DPLASMA_LU_CHUNKS=1
run gather_xr DPLASMA_LU_PANEL=gather DPLASMA_LU_XROWS=allreduce
run dist DPLASMA_LU_PANEL=dist
exit 0
