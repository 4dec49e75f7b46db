#!/usr/bin/env python3
"""tools/pmc_traffic.py -- HBM traffic per step from tools/pmc.sh output.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half of the bytes of wide streaming reads (128-B
requests tallied as 64 B), so reads are doubled; WRITE_SIZE is exact for
16-B stores.  Calibration check on the build: pass A's only reads are the
160 MB key stream, raw FETCH_SIZE 78.2 MiB -> x2 = 160 MB.  Other access
widths (the probe's random byte reads) are uncalibrated: the raw figures are
kept beside the corrected ones.

usage: python tools/pmc_traffic.py gpurun_out/pmc profiles/pmc_traffic.json single [launches_per_step]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out, workload = sys.argv[1], sys.argv[2], sys.argv[3]
launches_per_step = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
KERNELS = ("hash_var", "bloom_bin", "bloom_tile", "bloom_probe_multi", "pb_desc", "pb_hist", "pb_rows", "pb_scan",
           "pb_colsum", "pb_plan", "pb_starts",
           "pb_scatter", "pb_bin", "pb_tile", "pb_gather")
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        kern = next((n for n in KERNELS if n in k), None)
        if kern:
            acc[kern][row["Counter_Name"]].append(float(row["Counter_Value"]))
per = {}
total = 0.0
for kern, cs in acc.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * launches_per_step
    write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024 * launches_per_step
    e = {"fetch_bytes_raw": round(fetch), "read_bytes_corrected": round(2 * fetch),
         "write_bytes": round(write), "hbm_bytes": round(2 * fetch + write)}
    for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum"):
        if c in cs:
            e[c] = round(sum(cs[c]) / len(cs[c]) * launches_per_step)
    per[kern] = e
    total += 2 * fetch + write
d = {}
if os.path.exists(out):
    d = json.load(open(out))
if workload == "probe":  # the probe step is the pb_* pipeline; the builds in its setup are not part of it
    per = {k: v for k, v in per.items() if k.startswith("pb_") or k == "bloom_probe_multi"}
    total = sum(v["hbm_bytes"] for v in per.values())
d[workload] = {"hbm_bytes_per_build": round(total), "per_kernel": per,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; reads x2 (gfx950)"}
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d[workload], indent=1))
