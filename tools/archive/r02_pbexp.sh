#!/bin/bash
# tools/r02_pbexp.sh -- diagnostics build: P2 (pb_tile_kernel) time without
# its answer stores / bitmap loads / entry loads (wrong answers; timing only).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r02/pbexp}
mkdir -p "$OUT"
export TMPDIR=/tmp
for e in 0 1 2 4 7; do
  ADL_BLOOM_LIB=$PWD/adlsm-tree_amd/lib_stamps/libadlbloom.so ADL_PB_EXP=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/e$e" -o run --output-format csv -- \
    python3 bench.py --workload probe --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/e$e.log" 2>&1 || exit $?
  echo "exp=$e $(grep pb_tile "$OUT/e$e/run_kernel_stats.csv" | awk -F'",' '{print $2}' | cut -d, -f3)"
done
