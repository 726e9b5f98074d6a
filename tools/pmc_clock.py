#!/usr/bin/env python3
"""Per-dispatch effective clock and MFMA utilisation from a rocprofv3 --pmc CSV that holds
GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md: DVFS give-back).

clock = GRBM_GUI_ACTIVE / 8 XCDs / wall;  mfma util = MFMA_BUSY / (1024 SIMDs * clock * wall)."""
import csv
import sys
from collections import defaultdict

d = defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    key = (r["Dispatch_Id"], r["Kernel_Name"][:70])
    d[key][r["Counter_Name"]] = float(r["Counter_Value"])
    d[key]["wall"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for (did, name), v in sorted(d.items(), key=lambda x: int(x[0][0])):
    if v["wall"] < 1e-3 or "GRBM_GUI_ACTIVE" not in v:
        continue
    clk = v["GRBM_GUI_ACTIVE"] / 8 / v["wall"]
    util = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * clk * v["wall"])
    nm = v.get("SQ_INSTS_MFMA", 0)
    print(f"{did:>4} {v['wall'] * 1e3:8.2f} ms  clock {clk / 1e9:5.2f} GHz  mfma-busy {util * 100:5.1f}%  "
          f"mfma-insts {nm:.3g}  {name}")
