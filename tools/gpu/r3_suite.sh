#!/bin/bash
# Full GPU suite (one process, per-test timeout), smoke(), then the driver's default bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_suite_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3_suite_tests.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_suite_smoke.log 2>&1 || { cat gpurun_out/r3_suite_smoke.log; exit 1; }
tail -1 gpurun_out/r3_suite_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r3_suite_bench.log 2>&1
rc=$?; grep -E "TIME|metric" gpurun_out/r3_suite_bench.log | cut -c1-400; exit $rc
