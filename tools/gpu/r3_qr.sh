#!/bin/bash
# QR with the reference-pinned trees on one MI355X: GPU QR tests, then DGEQRF 32k/64k NB=256 flat vs
# HQR greedy domains of a tiles (a=-1 -> the reference's default 4), reference auto domino.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/r3_qr.log; : > $out
timeout -k 10 400 python -u -m pytest tests/test_qr.py tests/test_qrtree_parity.py -x -q -m gpu --timeout 150 \
    --timeout-method thread > gpurun_out/r3_qr_tests.log 2>&1 || { tail -30 gpurun_out/r3_qr_tests.log; exit 1; }
tail -2 gpurun_out/r3_qr_tests.log >> $out
run() { echo "== $*" >> $out; timeout -k 10 300 python tools/bench_algo.py "$@" >> $out 2>&1 || { tail -20 $out; exit 1; }; }
run geqrf -N 32768 --nb 256 --ib 32 --runs 2
for A in -1 8 16; do run geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a $A; done
run geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 8 --qr-tsrr 1
run geqrf -N 65536 --nb 256 --ib 32 --runs 1
run geqrf -N 65536 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16
grep -v amdgpu.ids $out
