#!/bin/bash
# r4 batch 30: round-end checks on a fresh MI355X after the last changes (full GPU suite, smoke, the driver's bench
# command), plus the LU-QR / HQR / DGETRF headline numbers of this round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b30
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|smoke" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python bench.py --steps 20 --warmup 5 || exit 1
grep -E '^\{' $O/bench.log | cut -c1-400
step luqr32k 300 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step hqr64k_a16 300 python tools/bench_algo.py geqrf -N 65536 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16 || exit 1
step geqrf64k_flat 300 python tools/bench_algo.py geqrf -N 65536 --nb 256 --ib 32 --runs 1 || exit 1
exit 0
