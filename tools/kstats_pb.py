#!/usr/bin/env python3
"""tools/kstats_pb.py -- the pb_* kernels' average times (us) and call counts
from a rocprofv3 --stats output directory.  usage: kstats_pb.py DIR"""
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    print(" ".join("%s=%.0f/%s" % (r["Name"][r["Name"].index("pb_"):].split("(")[0].split("<")[0], float(r["AverageNs"])/1e3, r["Calls"]) for r in csv.DictReader(open(f)) if "pb_" in r["Name"]))
