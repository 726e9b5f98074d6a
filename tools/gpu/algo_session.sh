#!/bin/bash
# secondary-metric timings on one MI355X: SUMMA DGEMM 32k, QR (flat + HQR), LU variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { timeout -k 10 ${T:-240} python tools/bench_algo.py "$@" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/algo.log; return ${PIPESTATUS[0]}; }
: > gpurun_out/algo.log
run gemm -N ${NG:-32768} --nb 512 --runs 2 || exit $?
run geqrf -N ${NQ:-16384} --nb 256 --ib 32 --runs 2 || exit $?
run geqrf -N ${NQ:-16384} --nb 256 --ib 32 --tree hqr --runs 2 || exit $?
run getrf_nopiv -N ${NL:-16384} --nb 512 --runs 2 || exit $?
run getrf_1d -N ${NL:-16384} --nb 512 --runs 2 || exit $?
run getrf_ptgpanel -N ${NL:-16384} --nb 512 --runs 2 || exit $?
run getrf_incpiv -N ${NL:-16384} --nb 256 --ib 32 --runs 2 || exit $?
exit 0
