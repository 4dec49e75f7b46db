#!/bin/bash
# tools/r03_probe2.sh -- probe tests, an A/B of the probe's K2 scan, and a
# rocprofv3 kernel trace of the probe bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_probe2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py \
  -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
AB="ADL_PB_OLDSCAN=1|ADL_PB_NEWSCAN=1" REPS=2 STEPS=5 BENCH_ARGS="--workload probe" timeout -k 10 600 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab_probe_scan.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --workload probe --no-cpu-baseline --no-e2e > "$OUT/prof_probe_bench.json" 2> "$OUT/prof_probe.err" || exit 1
find "$OUT/prof_probe" -name "*kernel_stats.csv" -exec cp {} "$OUT/probe_kernel_stats.csv" \;
