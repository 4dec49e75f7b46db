#!/bin/bash
# tools/r02_final.sh -- round-2 evidence in one GPU call: the GPU test suite,
# smoke(), the read-path latency bench, every bench workload (with CPU
# baselines) and a rocprofv3 kernel trace of the headline bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
step readpath
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --bench > "$OUT/readpath_bench.json" 2> "$OUT/readpath_bench.err" || exit 1
cat "$OUT/readpath_bench.json"
step bench_all
bash tools/bench_all.sh || exit 1
cp gpurun_out/bench_all.jsonl "$OUT/bench_all.jsonl"
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit 1
f=$(ls "$OUT"/prof/*kernel_stats.csv "$OUT"/prof/*/*kernel_stats.csv 2>/dev/null | head -1); echo "stats: $f"
exit 0
