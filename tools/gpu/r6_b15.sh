#!/bin/bash
# r6 batch 15: kernel trace of HQR replay rank 0 (2x4 64k NB=256 a=0, 16 hw queues)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b15
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== trace HQR replay rank 0" | tee -a $O/summary.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o rank0 -- \
  python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0 --bw 65 --lat 10 > $O/rp.log 2>&1 \
  || { tail -30 $O/rp.log | tee -a $O/summary.log; exit 1; }
grep -E "^rank" $O/rp.log | tee -a $O/summary.log
exit 0
