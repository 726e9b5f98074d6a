#!/bin/bash
# r6 batch 1: round-6 start check -- full GPU test suite, smoke, bench (driver command)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b1
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== gpu suite" | tee -a $O/summary.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "rc=$rc" | tee -a $O/summary.log
tail -5 $O/suite.log | tee -a $O/summary.log
[ $rc -eq 0 ] || exit 1
echo "== smoke" | tee -a $O/summary.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 | tee -a $O/summary.log
echo "== bench" | tee -a $O/summary.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -2 $O/bench.log | tee -a $O/summary.log
exit 0
