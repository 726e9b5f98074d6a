#!/bin/bash
# r5 batch 43: DGETRF look-ahead revisited with the tagged-granule panel kernel (32k / 64k; BW 64 vs 32)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b43
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1 N=$2; shift 2
  echo "== $name N=$N" | tee -a $O/summary.log
  env "$@" timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${name}_$N.log 2>&1
  local rc=$?
  grep TIME $O/${name}_$N.log | tail -1 | cut -c1-140 | tee -a $O/summary.log
  return $rc
}
for N in 32768 65536; do
  run base $N DPLASMA_LU_LOOKAHEAD=0 || exit 1
  run la64 $N DPLASMA_LU_LOOKAHEAD=1 || exit 1
  run la32 $N DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BW=32 || exit 1
  run bw32 $N DPLASMA_LU_LOOKAHEAD=0 DPLASMA_LU_BW=32 || exit 1
done
exit 0
