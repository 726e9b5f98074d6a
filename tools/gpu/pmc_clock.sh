#!/bin/bash
# effective clock (GRBM_GUI_ACTIVE/8/wall) + MFMA busy of our DGEMM vs the vendor DGEMM
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
VENDOR=1 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA -f csv -d $R/gpurun_out/pmc -o clk${N:-8192} -- python3 $R/tools/gpu/gemm_only.py ${N:-8192} 2 > $R/gpurun_out/pmc/clk.txt 2>&1
rc=$?; tail -1 $R/gpurun_out/pmc/clk.txt; exit $rc
