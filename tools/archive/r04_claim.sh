#!/bin/bash
# tools/r04_claim.sh -- pass A's claim layout (ADL_BLOOM_CLAIM=1: fixed
# per-tile slots claimed with one ds_add_rtn, no count pass or scan) against
# the chunk/table build, 2 interleaved reps on the headline, var-len and
# compaction workloads (each line's parity checked by bench.py), then the
# claim parity tests.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04cl
mkdir -p $OUT
bl() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-compaction-strong \
    ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']), flush=True)"
}
for rep in 1 2; do
  bl "single base" X=0 || exit 1
  bl "single claim" ADL_BLOOM_CLAIM=1 || exit 1
  bl "single claim slack115 sigma3" ADL_BLOOM_CLAIM=1 ADL_BLOOM_CLAIM_SLACK=115 ADL_BLOOM_CLAIM_SIGMA=3 || exit 1
done
for rep in 1 2; do
  BENCH_ARGS="--workload varlen" bl "varlen base" X=0 || exit 1
  BENCH_ARGS="--workload varlen" bl "varlen claim" ADL_BLOOM_CLAIM=1 || exit 1
  BENCH_ARGS="--workload compaction --steps 10" bl "compaction base" X=0 || exit 1
  BENCH_ARGS="--workload compaction --steps 10" bl "compaction claim" ADL_BLOOM_CLAIM=1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_claim.py > $OUT/parity.log 2>&1
rc=$?; echo "claim parity: $(tail -1 $OUT/parity.log)"; exit $rc
