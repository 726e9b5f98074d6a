#!/bin/bash
# DGEQRF split-K target sweep (DPLASMA_QR_SPLIT_WG: output workgroups per W = V^T C launch before the
# reduction dimension is split into partials) at 16k / 32k, NB=256 IB=32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/qr_split.log
: > $out
for N in 16384 32768; do
  for W in ${WGS:-128 256 512 1024 2048}; do
    echo "N=$N SPLIT_WG=$W" >> $out
    DPLASMA_QR_SPLIT_WG=$W timeout -k 10 200 python tools/bench_algo.py geqrf -N $N --nb 256 --ib 32 --runs 2 >> $out 2>&1 \
        || { tail -20 $out; exit 1; }
  done
done
grep -E "^N=|TIME" $out
