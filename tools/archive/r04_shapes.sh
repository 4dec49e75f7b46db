#!/bin/bash
# tools/r04_shapes.sh -- the bucketed build against the chunk/table build on the
# other build workloads (compaction, varlen), interleaved, plus the 2-rank test.
set -u
cd "$(dirname "$0")/.."
bl() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-compaction-strong --no-e2e --no-cpu-baseline \
    ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']))"
}
for rep in 1 2; do
  for wl in compaction varlen; do
    BENCH_ARGS="--workload $wl" bl "$wl bk " ADL_BLOOM_BK=1
    BENCH_ARGS="--workload $wl" bl "$wl old" ADL_BLOOM_BK=0
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_gpu_multirank.py 2>&1 | tail -2
