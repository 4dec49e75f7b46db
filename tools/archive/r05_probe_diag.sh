#!/bin/bash
# tools/r05_probe_diag.sh -- where the binned probe's time goes: rocprofv3
# kernel stats of the probe bench under the diagnostics build's ADL_PB_EXP
# switches (8 no hashing, 16 no hash-run stores, 32 no place stores; 1 no
# answer stores, 2 no bitmap loads, 4 no entry loads in pb_tile).  Wrong
# answers by design; only the per-kernel times are read.  TAG names gpurun_out/.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
export ADL_BLOOM_LIB=adlsm-tree_amd/lib_stamps/libadlbloom.so
for e in ${EXPS:-0 8 16 32 1 2 4}; do
  echo "=== ADL_PB_EXP=$e ($(date +%T))"
  ADL_PB_EXP=$e timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/e$e" -o run --output-format csv -- \
    python3 bench.py --workload probe --steps 6 --warmup 2 --no-e2e --no-cpu-baseline > "$OUT/e$e.json" 2> "$OUT/e$e.err" || exit $?
  python3 - "$OUT/e$e" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "pb_" in n:
            print("  %-14s %8.1f us x %s" % (n.split("(")[0].split("::")[-1].replace("void ", "")[:14], float(r["AverageNs"]) / 1e3, r["Calls"]))
PY
done
