#!/bin/bash
# r6 batch 32: rocprofv3 kernel stats of one DGETRF 64k (new one-process defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r6b32
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof --output-format csv -o getrf -- python $R/tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
grep TIME $O/run.log | tail -1 | cut -c1-140
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} n={int(r["Calls"]):6d} tot={float(r["TotalDurationNs"])/1e6:9.1f}ms avg={float(r["AverageNs"])/1e3:9.1f}us {100*float(r["TotalDurationNs"])/tot:6.2f}%')
PY
