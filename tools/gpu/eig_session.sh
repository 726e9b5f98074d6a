#!/bin/bash
# Eigen/SVD pipeline on one MI355X: GPU tests, then timings of herbt / heev / ge2gb.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_eigen.py -m gpu -x -q > gpurun_out/eig_tests.log 2>&1 || { tail -30 gpurun_out/eig_tests.log; exit 1; }
tail -3 gpurun_out/eig_tests.log
for args in "herbt -N 8192 --nb 256 --ib 32" "heev -N 4096 --nb 256 --ib 32" "gebrd_ge2gb -N 8192 --nb 256 --ib 32" "herbt -N 8192 --nb 128 --ib 32"; do
  timeout -k 10 300 python tools/bench_algo.py $args --runs 2 >> gpurun_out/eig_bench.log 2>&1 || { tail -20 gpurun_out/eig_bench.log; exit 1; }
done
cat gpurun_out/eig_bench.log
