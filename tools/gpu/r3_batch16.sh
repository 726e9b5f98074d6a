#!/bin/bash
# examples/native_dist_example.c: 1 rank (one-process engine) at 32k and 2 ranks sharing the GPU at 8k (file transport).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
gcc -O2 -o /tmp/nde examples/native_dist_example.c -Icapi/include -Ldplasma_amd/lib -ldplasma -lm -Wl,-rpath,$PWD/dplasma_amd/lib || exit 1
timeout -k 10 200 /tmp/nde 32768 512 1 > gpurun_out/b16_w1.log 2>&1 || { cat gpurun_out/b16_w1.log; exit 1; }
cat gpurun_out/b16_w1.log
RDV=$(mktemp -d)
export DPLASMA_NATIVE_RDV=$RDV DPLASMA_NATIVE_TRANSPORT=file DPLASMA_NATIVE_TIMEOUT=100 WORLD_SIZE=2 LOCAL_RANK=0
RANK=0 timeout -k 10 200 /tmp/nde 8192 512 2 > gpurun_out/b16_w2_r0.log 2>&1 &
p0=$!
RANK=1 timeout -k 10 200 /tmp/nde 8192 512 2 > gpurun_out/b16_w2_r1.log 2>&1 &
p1=$!
wait $p0; r0=$?; wait $p1; r1=$?
cat gpurun_out/b16_w2_r0.log; echo "rc $r0 $r1"
[ $r0 -eq 0 ] && [ $r1 -eq 0 ]
