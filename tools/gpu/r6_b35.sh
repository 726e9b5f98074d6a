#!/bin/bash
# r6 batch 35: QR panel kernel rows per workgroup (DPLASMA_QP_RMAX) on tall panels, with GMIN 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b35
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "r0:DPLASMA_QP_GMIN=8" "r128:DPLASMA_QP_GMIN=8 DPLASMA_QP_RMAX=128" "r64:DPLASMA_QP_GMIN=8 DPLASMA_QP_RMAX=64" "r32:DPLASMA_QP_GMIN=8 DPLASMA_QP_RMAX=32"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  echo "== $tag $e" | tee -a $O/summary.log
  env $e timeout -k 10 200 python tools/gpu/qr_panel_probe.py > $O/$tag.log 2>&1 || { tail -8 $O/$tag.log; exit 1; }
  grep "^M=" $O/$tag.log | cut -c1-100 | tee -a $O/summary.log
done
exit 0
