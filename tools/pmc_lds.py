#!/usr/bin/env python3
"""tools/pmc_lds.py -- the LDS bound of the build passes from a rocprofv3 PMC
pass of tools/pmc.sh whose group holds SQ_INSTS_LDS, SQ_LDS_IDX_ACTIVE,
SQ_LDS_BANK_CONFLICT, SQ_ACTIVE_INST_LDS, SQ_WAIT_INST_LDS and GRBM_GUI_ACTIVE.

MI355X_MICROARCH.md §LDS: SQ_LDS_IDX_ACTIVE counts all LDS-array cycles and
SQ_LDS_BANK_CONFLICT the extra cycles of bank conflicts (summed over the
CUs).  Per build kernel, averaged over its launches: LDS instructions, array
cycles, conflict cycles, their ratio, and the LDS array's busy fraction
(array cycles / (256 CUs x kernel cycles), the clock from GRBM_GUI_ACTIVE / 8
XCDs / the dispatch's duration in the same pass).  Written into
profiles/pmc_traffic.json[workload]["lds"], keyed like ["alu"]; bench.py
reports it as roofline.lds.

usage: python tools/pmc_lds.py gpurun_out/pmc_lds profiles/pmc_traffic.json single
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
PASS_OF = {"hash_var": "hash_var_kernel", "bloom_bin": "bloom_bin_kernel", "bloom_tile": "bloom_tile_kernel"}
COUNTERS = ("SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS",
            "GRBM_GUI_ACTIVE")
CUS = 256

dur = {}
for f in glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True):
    p = f.split(os.sep + "p")[1].split(os.sep)[0]
    for row in csv.DictReader(open(f)):
        dur[(p, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])

per_dispatch = defaultdict(dict)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    p = f.split(os.sep + "p")[1].split(os.sep)[0]
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] in COUNTERS:
            d = per_dispatch[(p, row["Dispatch_Id"])]
            d["kernel"] = row["Kernel_Name"]
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])

acc = defaultdict(lambda: defaultdict(list))
for key, d in per_dispatch.items():
    short = next((s for s in PASS_OF if s in d["kernel"]), None)
    if not short or "SQ_LDS_IDX_ACTIVE" not in d:
        continue
    acc[short]["dur_ns"].append(dur.get(key, 0))
    for c in COUNTERS:
        if c in d:
            acc[short][c].append(d[c])

res = {}
for short, cs in acc.items():
    mean = {c: sum(v) / len(v) for c, v in cs.items() if v}
    clk = mean["GRBM_GUI_ACTIVE"] / 8 / mean["dur_ns"] if mean.get("GRBM_GUI_ACTIVE") and mean["dur_ns"] else None
    idx, conf = mean["SQ_LDS_IDX_ACTIVE"], mean.get("SQ_LDS_BANK_CONFLICT", 0.0)
    e = {"launches": len(cs["SQ_LDS_IDX_ACTIVE"]), "lds_insts": round(mean.get("SQ_INSTS_LDS", 0)),
         "array_cycles": round(idx), "conflict_cycles": round(conf),
         "conflict_frac": round(conf / idx, 4) if idx else None,
         "dur_us_profiled": round(mean["dur_ns"] / 1e3, 2), "clock_ghz": round(clk, 3) if clk else None,
         "active_inst_lds": round(mean.get("SQ_ACTIVE_INST_LDS", 0)), "wait_inst_lds": round(mean.get("SQ_WAIT_INST_LDS", 0))}
    if clk:
        e["array_busy_frac"] = round(idx / (CUS * mean["dur_ns"] * clk), 4)
    res[PASS_OF[short]] = e
d = json.load(open(out)) if os.path.exists(out) else {}
d.setdefault(workload, {})["lds"] = res
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
