#!/bin/bash
# r6 batch 12: DTR (push scheduler) at one vs two workgroups per CU after the co-residency fix, 16k / 32k / 64k,
# against the stream engine; every run residual-checked by bench.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b12
mkdir -p $O
export PYTHONUNBUFFERED=1
for N in 16384 32768 65536; do
  S=10; [ $N -ge 32768 ] && S=5; [ $N -ge 65536 ] && S=4
  for WG in 256 512; do
    echo "== N=$N dtr WG=$WG" | tee -a $O/summary.log
    DPLASMA_POTRF_ENGINE=dtr DPLASMA_DTR_WG=$WG timeout -k 10 300 python bench.py -N $N --steps $S --warmup 2 > $O/b_${N}_$WG.log 2>&1 \
      || { tail -5 $O/b_${N}_$WG.log | tee -a $O/summary.log; exit 1; }
    grep -o '"value": [0-9.]*\|"check": [a-z]*\|"engine": "[a-z]*"' $O/b_${N}_$WG.log | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  done
  echo "== N=$N stream engine" | tee -a $O/summary.log
  DPLASMA_POTRF_ENGINE=stream timeout -k 10 300 python bench.py -N $N --steps $S --warmup 2 > $O/b_${N}_s.log 2>&1 \
    || { tail -5 $O/b_${N}_s.log | tee -a $O/summary.log; exit 1; }
  grep -o '"value": [0-9.]*\|"check": [a-z]*\|"engine": "[a-z]*"' $O/b_${N}_s.log | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
done
exit 0
