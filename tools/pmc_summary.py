#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSVs per kernel: python tools/pmc_summary.py CSV [CSV ...] [--match k_gemm]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
agg = defaultdict(lambda: defaultdict(float))
for f in args:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        agg[k[:90]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:28s} {x:.4g}")
    w = v.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_INST_CYCLES_VMEM"):
            if c in v:
                print(f"   {c}/WAVE_CYCLES = {v[c] / w:.3f}")
