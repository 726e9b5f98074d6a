#!/bin/bash
# DGETRF look-ahead with the bulk update capped (DPLASMA_LU_REST_CAP workgroups) so the next panel's persistent
# kernel (lds 64 / lds 32 / reg) co-resides beside it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > gpurun_out/b14_${N}_$tag.log 2>&1 \
    || { echo "$tag failed"; tail -5 gpurun_out/b14_${N}_$tag.log; exit 1; }
  echo "N=$N $tag: $(grep TIME gpurun_out/b14_${N}_$tag.log | tail -1 | cut -c1-120)"
}
for N in 32768 65536; do
  run base DPLASMA_LU_LOOKAHEAD=0
  run reg_la_cap256 DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BLOCK=reg DPLASMA_LU_REST_CAP=256
  run reg_la_cap384 DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BLOCK=reg DPLASMA_LU_REST_CAP=384
  run bw32_la_cap256 DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BW=32 DPLASMA_LU_REST_CAP=256
  run lds_la_cap256 DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_REST_CAP=256
done
exit 0
