#!/bin/bash
# r6 batch 41: 2x4 grid emulation with one workgroup per CU (the emulation's default now), 32k / 64k, checked
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b41
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for N in 32768 65536; do
  timeout -k 10 500 python -u tools/emulate_potrf.py -N $N --grid 2x4 --reps 2 --check > $O/e_$N.log 2>&1 || { tail -10 $O/e_$N.log; exit 1; }
  grep -E "EMUL|residual" $O/e_$N.log
done
exit 0
