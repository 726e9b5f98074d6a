#!/bin/bash
# QR engine session on one MI355X: panel-kernel + engine tests, then DGEQRF timings (flat / HQR),
# then a kernel-trace profile of one 16k factorisation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_qr.py -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "${QR_TESTS:-panel or gpu_qr or gpu_hqr or gpu_gels or gpu_unmqr}" 2>&1 | tail -25 || exit $?
run() { timeout -k 10 ${T:-240} python tools/bench_algo.py "$@" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/qr.log; return ${PIPESTATUS[0]}; }
: > gpurun_out/qr.log
for n in ${NQS:-8192 16384 32768}; do
  run geqrf -N $n --nb 256 --ib 32 --runs 2 || exit $?
done
run geqrf -N ${NQ:-16384} --nb 256 --ib 32 --tree hqr --runs 2 || exit $?
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_qr -o run -- \
    python tools/bench_algo.py geqrf -N ${NQ:-16384} --nb 256 --ib 32 --runs 1 > gpurun_out/prof_qr.log 2>&1 || exit $?
fi
exit 0
