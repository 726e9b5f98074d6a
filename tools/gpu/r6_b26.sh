#!/bin/bash
# r6 batch 26: DTR idle workgroups skip the ring scan while no task completed (DPLASMA_DTR_SCANSKIP) -- correctness
# (DTR GPU tests), 16k trace, 16k / 32k / 64k against the full rescan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b26
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_potrf_dtr.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/gpu/dtr_trace_run.py 16384 gpurun_out/dtr16k_skip.npz > $O/trace16k.log 2>&1 || { tail -20 $O/trace16k.log; exit 1; }
head -3 $O/trace16k.log | tail -2; grep -A3 "^POTRF(1)" $O/trace16k.log
for cfg in "skip:" "noskip:DPLASMA_DTR_SCANSKIP=0" "skip2:" "noskip2:DPLASMA_DTR_SCANSKIP=0"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  echo "== $tag $e" | tee -a $O/summary.log
  env $e timeout -k 10 300 python tools/gpu/dtr_bench.py --engine dtr --reps 4 16384 32768 65536 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  grep TIME $O/$tag.log | cut -c1-150 | tee -a $O/summary.log
done
exit 0
