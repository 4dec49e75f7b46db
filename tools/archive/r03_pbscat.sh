#!/bin/bash
# tools/r03_pbscat.sh -- diagnostics build: K3 (pb_scatter_kernel) time without
# its hashing / run stores / place stores (wrong answers; timing only).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_pbscat}
mkdir -p "$OUT"
export TMPDIR=/tmp
for e in 0 8 16 32 56; do
  ADL_BLOOM_LIB=$PWD/adlsm-tree_amd/lib_stamps/libadlbloom.so ADL_PB_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/e$e" -o run --output-format csv -- \
    python3 bench.py --workload probe --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/e$e.log" 2>&1 || exit $?
  echo "exp=$e $(grep pb_scatter "$OUT/e$e/run_kernel_stats.csv" | awk -F'",' '{print $2}' | cut -d, -f3)"
done
