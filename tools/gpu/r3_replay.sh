#!/bin/bash
# Rank replay of the 2x4 (and 2x1, 4x1) distributed Cholesky at N=65536 NB=512 on one GPU
# (tools/replay_potrf.py), over the distributed schedule knobs.  REPLAY_CFGS: ';'-separated env sets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${REPLAY_OUT:-replay.log}
: > $OUT
GRID=${REPLAY_GRID:-2x4}
RANKS=${REPLAY_RANKS:-0,7}
N=${REPLAY_N:-65536}
IFS=';' read -ra CFGS <<< "${REPLAY_CFGS:-DPLASMA_POTRF_DEFER=2}"
for cfg in "${CFGS[@]}"; do
  echo "=== $GRID N=$N ranks=$RANKS $cfg ${REPLAY_ARGS}" | tee -a $OUT
  env $cfg timeout -k 10 240 python tools/replay_potrf.py -N $N --grid $GRID --ranks $RANKS --steps 1 \
      ${REPLAY_ARGS} >> $OUT 2>&1
  rc=$?
  tail -1 $OUT | cut -c1-400
  [ $rc -ne 0 ] && { tail -30 $OUT; exit $rc; }
done
exit 0
