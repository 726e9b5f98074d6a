#!/bin/bash
# DGETRF (partial pivoting) tile-size sweep on one MI355X: the trailing update's k-run is NB, so a
# wider tile moves the bulk GEMM to its large-k rate; the panel's per-column latency is paid N times
# whatever NB is.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/lu_nb.log
: > $out
for N in 32768 65536; do
  for NB in ${NBS:-512 768 1024}; do
    echo "N=$N NB=$NB" >> $out
    timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb $NB --runs 2 >> $out 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -20 $out; exit $rc; }
  done
done
grep -E "^N=|TIME" $out
