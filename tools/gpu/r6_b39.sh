#!/bin/bash
# r6 batch 39: 2x4 grid emulation of the distributed DTR -- 32k with the round-5 priority weights vs the current ones;
# 64k current
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b39
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
em() { local tag=$1 n=$2; shift 2; env "$@" timeout -k 10 400 python -u tools/emulate_potrf.py -N $n --grid 2x4 --reps 2 > $O/$tag.log 2>&1 || { tail -10 $O/$tag.log; exit 1; }; echo "$tag: $(grep EMUL $O/$tag.log)"; }
em w_r5_32k 32768 DPLASMA_DTR_BL_W=75,65,175,300
em w_cur_32k 32768 DPLASMA_DTR_NAP=0
em w_scanoff_32k 32768 DPLASMA_DTR_SCANSKIP=0
em w_cur_64k 65536 DPLASMA_DTR_NAP=0
em w_r5_64k 65536 DPLASMA_DTR_BL_W=75,65,175,300
exit 0
