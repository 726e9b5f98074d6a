#!/bin/bash
# Kernel trace of one replayed rank of the distributed Cholesky (tools/replay_potrf.py).
# env: RP_RANK (0), RP_ARGS (replay args), RP_TAG (output name); DPLASMA_* knobs exported by the caller.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
TAG=${RP_TAG:-replay}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/$TAG -o $TAG -- \
    python3 $R/tools/replay_potrf.py -N ${RP_N:-65536} --grid ${RP_GRID:-2x4} --ranks ${RP_RANK:-0} --steps 1 $RP_ARGS \
    > $R/gpurun_out/$TAG.log 2>&1
rc=$?; tail -1 $R/gpurun_out/$TAG.log | cut -c1-300; exit $rc
