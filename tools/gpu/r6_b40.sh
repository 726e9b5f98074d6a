#!/bin/bash
# r6 batch 40: 2x4 emulation A/B -- the round-5 DTR kernel (a65528d dtr.hip + its headers, linked with today's other
# kernels) against today's, same host code and box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=gpurun_out/r6b40
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
em() { local tag=$1 n=$2; shift 2; env "$@" timeout -k 10 400 python -u tools/emulate_potrf.py -N $n --grid 2x4 --reps 2 > $O/$tag.log 2>&1 || { tail -10 $O/$tag.log; exit 1; }; echo "$tag: $(grep EMUL $O/$tag.log)"; }
em r5k_32k 32768 DPLASMA_KERNELS_LIB=$R/dplasma_amd/lib/libdplasma_kernels_r5dtr.so
em cur_32k 32768 DPLASMA_DTR_NAP=0
em r5k_64k 65536 DPLASMA_KERNELS_LIB=$R/dplasma_amd/lib/libdplasma_kernels_r5dtr.so
exit 0
