#!/bin/bash
# r5 batch 33: push-scheduled DTR (k_dtr_q): GPU tests, speed vs the list scheduler, repeat checks, 16k trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b33
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== gpu tests (dtr)" | tee -a $O/summary.log
timeout -k 10 300 python -u -m pytest tests/test_potrf_dtr.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "rc=$rc" | tee -a $O/summary.log
tail -3 $O/tests.log | tee -a $O/summary.log
[ $rc -eq 0 ] || exit 1
perf() {
  echo "== $1" | tee -a $O/summary.log
  shift
  env "$@" timeout -k 10 240 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
}
perf queue_256 DPLASMA_DTR_SCHED=queue
perf queue_512 DPLASMA_DTR_SCHED=queue DPLASMA_DTR_WG=512
echo "== repeat queue 32k" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 12 > $O/rep.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "False|FAILED|counters" $O/rep.log | cut -c1-300 | tee -a $O/summary.log
echo "== trace queue 16k" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_trace_run.py 16384 $O/trace16k_q.npz > $O/trace16k.log 2>&1
head -8 $O/trace16k.log | tee -a $O/summary.log
timeout -k 10 300 python tools/emul_critical.py $O/trace16k_q.npz 1 30 > $O/crit16k.log 2>&1
head -40 $O/crit16k.log | tee -a $O/summary.log
echo "== dist rehearsal queue 2 ranks 1x2 16k" | tee -a $O/summary.log
DPLASMA_DTR_SCHED=queue DPLASMA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 tools/gpu/dtr_dist_rehearsal.py 16384 1 3 > $O/reh12.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "run |DTR-DIST|Error|error" $O/reh12.log | head -8 | tee -a $O/summary.log
echo "== dist rehearsal queue 4 ranks 2x2 16k" | tee -a $O/summary.log
DPLASMA_DTR_SCHED=queue DPLASMA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29521 tools/gpu/dtr_dist_rehearsal.py 16384 2 3 > $O/reh22.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "run |DTR-DIST|Error|error" $O/reh22.log | head -8 | tee -a $O/summary.log
exit 0
