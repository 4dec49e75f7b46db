#!/bin/bash
# tools/r05_pmc.sh -- round 5 counters at the current code: every PMC pass of
# tools/pmc_all.sh (traffic, integer issue, LDS array / bank-conflict cycles)
# for the build workloads and the probe, then a kernel-trace --stats run of the
# headline bench.  TAG names the gpurun_out/ directory; the refreshed
# profiles/pmc_traffic.json comes back as gpurun_out/$TAG/pmc_traffic.json.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/pmc_all.sh "$OUT" ${WORKLOADS:-single compaction varlen probe} || exit $?
echo "=== stats ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-e2e --no-compaction-strong --no-cpu-baseline \
  > "$OUT/stats_bench.json" 2> "$OUT/stats_bench.err" || exit $?
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -c1-300 "$OUT/stats_bench.json"
