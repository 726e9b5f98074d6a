#!/bin/bash
# r4 batch 1: the tile-kernel flag race (stream-ordered init + ticket ids): potrf tile tests, then
# the headline bench under rocprofv3 --kernel-trace (the configuration that timed out in round 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b1
export PYTHONUNBUFFERED=1
python -c "import torch; print('torch', torch.__version__, torch.cuda.get_device_name(0))" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_tile_gpu.py \
  > gpurun_out/r4b1/tile_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4b1/tile_tests.log; echo "tile tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b1/prof -o potrf -- \
  python bench.py --steps 2 --warmup 1 > gpurun_out/r4b1/bench_prof.log 2>&1
rc=$?; grep -E '^\{|Error|error|info' gpurun_out/r4b1/bench_prof.log | head -5; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r4b1/bench.log 2>&1
rc=$?; tail -2 gpurun_out/r4b1/bench.log; echo "bench rc=$rc"
exit $rc
