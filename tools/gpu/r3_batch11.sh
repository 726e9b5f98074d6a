#!/bin/bash
# Multi-process native C ABI, ranks launched directly (per-rank logs, short timeouts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
gcc -O2 -o /tmp/tnd tests/capi/test_native_dist.c -Icapi/include -Ldplasma_amd/lib -ldplasma -lm -Wl,-rpath,$PWD/dplasma_amd/lib || exit 1
export DPLASMA_NATIVE_TRANSPORT=file DPLASMA_NATIVE_TIMEOUT=40 DPLASMA_NATIVE_DEBUG=1
for cfg in ${CFGS:-2:2 2:1 4:2}; do
  W=${cfg%:*}; P=${cfg#*:}; RDV=$(mktemp -d)
  pids=()
  for ((r=0; r<W; r++)); do
    timeout -k 5 90 /tmp/tnd $r $W $P $RDV > gpurun_out/b11_w${W}p${P}_r$r.log 2>&1 &
    pids+=($!)
  done
  rc=0; for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "world=$W P=$P rc=$rc"; for ((r=0; r<W; r++)); do grep -E "FAIL|passed|failed|diff" gpurun_out/b11_w${W}p${P}_r$r.log | tail -40; done
  [ $rc -ne 0 ] && exit $rc
done
exit 0
