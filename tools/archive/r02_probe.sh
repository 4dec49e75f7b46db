#!/bin/bash
# tools/r02_probe.sh -- binned probe: parity tests, the probe bench line, its rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py -m gpu -q -x -rf --timeout 300 --timeout-method thread > "$OUT/probe_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 "$OUT/probe_pytest.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload probe --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_probe2.log" 2>&1 || exit $?
grep '^{' "$OUT/bench_probe2.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])'
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe2" -o run --output-format csv -- \
  python3 bench.py --workload probe --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/rocprof_probe2.log" 2>&1 || exit $?
grep -E "pb_|bloom_probe" "$OUT/prof_probe2/run_kernel_stats.csv" | awk -F'",' '{n=$1; sub(/\(.*/,"",n); print n, $2}'
exit 0
