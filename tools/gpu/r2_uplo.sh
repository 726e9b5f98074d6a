#!/bin/bash
# DPOTRF lower vs upper on one MI355X (the reference's testing_zpotrf defaults to Upper), with check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/uplo.log
: > $out
for N in 16384 32768 65536; do
  for U in L U; do
    st=5; [ $N -eq 65536 ] && st=3
    echo "N=$N uplo=$U" >> $out
    timeout -k 10 240 python bench.py -N $N --uplo $U --steps $st --warmup 1 >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
grep -E "^N=|TIME|\"check\"" $out | sed 's/, "data".*"check": / check=/' | cut -c1-200
