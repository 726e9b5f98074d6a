#!/bin/bash
# r6 batch 24: device-decided LU-QR on several processes (two ranks sharing the GPU, gloo), + the LU-QR GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b24
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 \
  tools/gpu/luqr_dist_rehearsal.py 2048 256 2 > $O/rehearsal_2x1.log 2>&1 || { grep -v Gloo $O/rehearsal_2x1.log | tail -30; exit 1; }
grep -E "crit=|REHEARSAL" $O/rehearsal_2x1.log
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29632 \
  tools/gpu/luqr_dist_rehearsal.py 2048 256 2 > $O/rehearsal_2x2.log 2>&1 || { grep -v Gloo $O/rehearsal_2x2.log | tail -30; exit 1; }
grep -E "crit=|REHEARSAL" $O/rehearsal_2x2.log
timeout -k 10 400 python -u -m pytest tests/test_lu_qr.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
