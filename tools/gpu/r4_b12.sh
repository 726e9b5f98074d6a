#!/bin/bash
# r4 batch 12: the round-end checks -- full GPU test suite (one process, per-test timeout), smoke(), and the
# driver's bench command (20 timed steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b12
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?; tail -5 $O/gpu_suite.log; echo "suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; grep -E '^\{' $O/bench.log | cut -c1-400; echo "bench rc=$rc"
exit $rc
