#!/bin/bash
# r6 batch 34: QR panel kernel with a minimum workgroup count (DPLASMA_QP_GMIN) on short (TT / small TS) panels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b34
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for g in 0 4 8 16; do
  echo "== GMIN=$g" | tee -a $O/summary.log
  DPLASMA_QP_GMIN=$g timeout -k 10 200 python tools/gpu/qr_panel_probe.py > $O/g$g.log 2>&1 || { tail -8 $O/g$g.log; exit 1; }
  grep -A1 "^M=" $O/g$g.log | tee -a $O/summary.log
done
exit 0
