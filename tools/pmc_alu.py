#!/usr/bin/env python3
"""tools/pmc_alu.py -- SURVEY.md §8(d)'s secondary bound (integer issue) from a
rocprofv3 PMC pass of tools/pmc.sh whose group holds SQ_INSTS_VALU (plus
SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE).

Per build kernel, averaged over its launches: VALU wave-instructions, SALU and
LDS instructions, and the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs /
kernel duration from the same pass's kernel trace; MI355X_MICROARCH.md
'DVFS give-back').  Written into profiles/pmc_traffic.json[workload]["alu"],
keyed as bench.py's roofline.us_per_step ("bloom_bin_kernel" = pass A, which
for var-len keys includes the hashing pass; "bloom_tile_kernel" = pass B).
bench.py turns it into roofline.alu at the run's own kernel times.

usage: python tools/pmc_alu.py gpurun_out/pmc_alu profiles/pmc_traffic.json single
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
PASS_OF = {"hash_var": "bloom_bin_kernel", "bloom_bin": "bloom_bin_kernel", "bloom_tile": "bloom_tile_kernel"}
COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE")

# dispatch id -> (kernel, duration ns) from every pass's kernel trace
dur = {}
for f in glob.glob(os.path.join(root, "p*", "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        dur[(f.split(os.sep + "p")[1].split(os.sep)[0], row["Dispatch_Id"])] = (
            row["Kernel_Name"], int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))

# pass -> dispatch -> counter values
per_dispatch = defaultdict(dict)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    p = f.split(os.sep + "p")[1].split(os.sep)[0]
    for row in csv.DictReader(open(f)):
        if row["Counter_Name"] in COUNTERS:
            d = per_dispatch[(p, row["Dispatch_Id"])]
            d["kernel"] = row["Kernel_Name"]
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])

acc = defaultdict(lambda: defaultdict(list))  # pass key -> counter -> per-launch values
for key, d in per_dispatch.items():
    short = next((s for s in PASS_OF if s in d["kernel"]), None)
    if not short or "SQ_INSTS_VALU" not in d:
        continue
    kname, ns = dur.get(key, (None, 0))
    acc[short]["dur_ns"].append(ns)
    for c in COUNTERS:
        if c in d:
            acc[short][c].append(d[c])

res = {}
for short, cs in acc.items():
    n = len(cs["SQ_INSTS_VALU"])
    mean = {c: sum(v) / len(v) for c, v in cs.items() if v}
    e = {"launches": n, "valu_wave_insts": round(mean["SQ_INSTS_VALU"]),
         "salu_insts": round(mean.get("SQ_INSTS_SALU", 0)), "lds_insts": round(mean.get("SQ_INSTS_LDS", 0)),
         "dur_us_profiled": round(mean["dur_ns"] / 1e3, 2)}
    if mean.get("GRBM_GUI_ACTIVE") and mean["dur_ns"]:
        e["clock_ghz"] = round(mean["GRBM_GUI_ACTIVE"] / 8 / mean["dur_ns"], 3)
    tgt = PASS_OF[short]
    if tgt in res:  # var-len pass A = hashing pass + bin pass: instructions add, the clock is the bin pass's
        for k in ("valu_wave_insts", "salu_insts", "lds_insts", "dur_us_profiled"):
            res[tgt][k] = round(res[tgt][k] + e[k], 2)
        res[tgt].setdefault("parts", []).append(short)
    else:
        res[tgt] = dict(e, parts=[short])
d = json.load(open(out)) if os.path.exists(out) else {}
d.setdefault(workload, {})["alu"] = res
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
