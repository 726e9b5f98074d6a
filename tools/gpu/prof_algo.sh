#!/bin/bash
# kernel-trace profile of one bench_algo op: OP, N, NB, IB env
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out/pa
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/pa -o ${OP} -- python3 $R/tools/bench_algo.py ${OP} -N ${N:-16384} --nb ${NB:-512} --ib ${IB:-32} --runs 2 ${EXTRA} > $R/gpurun_out/pa/${OP}.log 2>&1
rc=$?; grep TIME $R/gpurun_out/pa/${OP}.log; exit $rc
