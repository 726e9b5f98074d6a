#!/bin/bash
# PMC counters (kernel-trace only, no sys/runtime trace) for the QR kernels at N=8192.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -f csv -d $R/gpurun_out/pmc_qr -o qr -- python3 $R/tools/bench_algo.py geqrf -N ${QR_N:-8192} --nb 256 --ib 32 --runs 1 > $R/gpurun_out/pmc_qr.log 2>&1
rc=$?; tail -3 $R/gpurun_out/pmc_qr.log; exit $rc
