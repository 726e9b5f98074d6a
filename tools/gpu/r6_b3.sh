#!/bin/bash
# r6 batch 3: w4 anomaly probe (tools/gpu/dtr_w4_queues.py) + the new GPU tests of the p2p LU interchanges
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b3
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== xrows kernels + 2/4-rank LU rehearsal (p2p interchanges on the GPU, gloo host side)" | tee -a $O/summary.log
timeout -k 10 600 python -u -m pytest tests/test_lu_xrows.py tests/test_gpu_lu_dist.py -m gpu -x -v --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -12 | tee -a $O/summary.log
[ $rc -eq 0 ] || exit 1
for w in 2 4; do
  echo "== w$w queue probe" | tee -a $O/summary.log
  env DPLASMA_DIST_BACKEND=gloo DPLASMA_DTR_WG=$((256 / w)) timeout -k 10 240 python -m torch.distributed.run \
    --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29700 + w)) tools/gpu/dtr_w4_queues.py 16384 \
    > $O/w$w.log 2>&1 || { tail -20 $O/w$w.log | tee -a $O/summary.log; exit 1; }
  grep "N=" $O/w$w.log | tee -a $O/summary.log
done
echo "== LU panel cross-rank hand-off probe (two emulated ranks on the two CU halves)" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/lu_xlat_probe.py 65536 2 32 64 96 112 > $O/xlat.log 2>&1 || { tail -20 $O/xlat.log | tee -a $O/summary.log; exit 1; }
grep -E "k=|N=" $O/xlat.log | tee -a $O/summary.log
exit 0
