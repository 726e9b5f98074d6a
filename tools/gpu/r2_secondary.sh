#!/bin/bash
# Secondary metrics of BASELINE.json on one MI355X: DGEMM 32k NB=512, DGETRF, DGEQRF / HQR, ZPOTRF.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/secondary.log; : > $out
run() { echo "== $*" >> $out; timeout -k 10 300 python tools/bench_algo.py "$@" 2>&1 | grep TIME >> $out || { cat $out; exit 1; }; }
run gemm -N 32768 --nb 512 --runs 2
run getrf_1d -N 32768 --nb 512 --runs 2
run getrf_1d -N 65536 --nb 512 --runs 1
run geqrf -N 32768 --nb 256 --ib 32 --runs 2
run geqrf -N 65536 --nb 256 --ib 32 --runs 1
run geqrf -N 32768 --nb 256 --ib 32 --tree hqr --qr-llvl 0 --qr-hlvl 0 --runs 2
run getrf_nopiv -N 32768 --nb 512 --runs 2
cat $out
