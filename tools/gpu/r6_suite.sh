#!/bin/bash
# r6: GPU test suite in two groups (GROUP=a: kernel-level files, b: the rest)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6suite
mkdir -p $O
export PYTHONUNBUFFERED=1
A="tests/test_gpu_kernels.py tests/test_potrf_tile_gpu.py tests/test_zgemm_gpu.py"
if [ "${GROUP:-a}" = a ]; then
  timeout -k 10 1080 python -u -m pytest $A -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider \
    > $O/a.log 2>&1; rc=$?
  tail -5 $O/a.log; exit $rc
fi
IGN=""
for f in $A; do IGN="$IGN --ignore=$f"; done
timeout -k 10 1080 python -u -m pytest tests $IGN -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  > $O/b.log 2>&1; rc=$?
tail -8 $O/b.log; exit $rc
