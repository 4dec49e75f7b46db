#!/bin/bash
# tools/r02_varhash.sh -- the length-sorted var-len hashing pass: var-len parity
# tests, the configs[2] full-size pin, bench --workload varlen with the pass on
# and off, and a rocprofv3 kernel trace of the var-len bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/varhash
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q -rf \
  --timeout 200 --timeout-method thread -k "varlen or zipf or config2 or murmur or appendix" > "$OUT/pytest.log" 2>&1
rc=$?; tail -n 5 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for vh in 1 0 1; do
  echo "=== bench VAR_HASH=$vh ($(date +%T))"
  ADL_BLOOM_VAR_HASH=$vh timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload varlen --no-cpu-baseline --no-e2e \
    > "$OUT/bench_$vh.log" 2>&1 || exit 1
  grep '^{' "$OUT/bench_$vh.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])'
done
echo "=== rocprof ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --workload varlen --no-cpu-baseline --no-e2e > "$OUT/prof_bench.log" 2>&1 || exit 1
f=$(ls "$OUT"/prof/*kernel_stats.csv "$OUT"/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cut -d, -f1-8 "$f" | head -12
exit 0
