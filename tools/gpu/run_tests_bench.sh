#!/bin/bash
# GPU session: kernel numerics tests, then benches.  Stops at the first GPU fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N_BENCH=${N_BENCH:-65536}
python -c "import torch; print('torch', torch.__version__, torch.cuda.get_device_name(0))"
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py -N 16384 --steps 2 --warmup 1 --check > gpurun_out/bench_16k.log 2>&1
rc=$?; cat gpurun_out/bench_16k.log; echo "bench16k rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py -N ${N_BENCH} --steps 2 --warmup 1 > gpurun_out/bench_full.log 2>&1
rc=$?; cat gpurun_out/bench_full.log; echo "bench rc=$rc"
exit $rc
