#!/usr/bin/env python3
"""tools/pmc_summary.py -- per-kernel averages of the rocprofv3 PMC passes
written by tools/pmc.sh (gpurun_out/pmc/p*/run_counter_collection.csv)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        short = ("bin" if "bloom_bin" in k else "tile" if "bloom_tile" in k else "hash_var" if "hash_var" in k
                 else k[:40])
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    if k not in ("bin", "tile", "hash_var"):
        continue
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
