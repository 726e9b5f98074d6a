#!/bin/bash
# Kernel stats of HQR (greedy domains a=4) DGEQRF 16k NB=256 on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/phqr -o p -- python3 $R/tools/bench_algo.py geqrf -N 16384 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a ${QA:--1} > $R/gpurun_out/phqr.log 2>&1
