#!/bin/bash
# PMC passes over one 8192^3 DGEMM (each pass its own run; <= 8 SQ counters per pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_IFETCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_FLAT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -f csv -d $R/gpurun_out/pmc -o gemm${N:-8192}_p$i -- python3 $R/tools/gpu/gemm_only.py ${N:-8192} 1 > $R/gpurun_out/pmc/log$i.txt 2>&1
  rc=$?; tail -1 $R/gpurun_out/pmc/log$i.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
