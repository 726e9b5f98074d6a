#!/bin/bash
# r6 batch 42: 2x4 32k grid emulation -- deferral depth and list order sweep (one workgroup per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b42
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "d2 --defer 2" "d3 --defer 3" "d4 --defer 4" "d2col --defer 2 --order column" "d4col --defer 4 --order column" "d1 --defer 1"; do
  set -- $cfg; tag=$1; shift
  timeout -k 10 300 python -u tools/emulate_potrf.py -N 32768 --grid 2x4 --reps 2 "$@" > $O/$tag.log 2>&1 || { tail -10 $O/$tag.log; exit 1; }
  echo "$tag: $(grep EMUL $O/$tag.log)"
done
exit 0
