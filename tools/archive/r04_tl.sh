#!/bin/bash
# tools/r04_tl.sh -- build tile size (ADL_BLOOM_TILE_LOG2; auto: 2^20-bit
# tiles) and pass B at two workgroups per CU (ADL_BLOOM_B_OCC=2: 64-VGPR
# kernels, half the segment batch, pipeline depth 4 or 6), each setting
# checked against the pins by bench.py; parity tests of the two-per-CU
# kernels first.  2 interleaved reps.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04t
mkdir -p $OUT
for tl in 18 19; do
  ADL_BLOOM_B_OCC=2 ADL_BLOOM_DEPTH=4 ADL_BLOOM_TILE_LOG2=$tl timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_parity.py -k "build" > $OUT/parity_occ2_tl$tl.log 2>&1
  rc=$?; echo "occ2 TL=$tl parity $(tail -1 $OUT/parity_occ2_tl$tl.log)"; [ $rc -eq 0 ] || exit $rc
done
bl() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-compaction-strong \
    ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']))"
}
for rep in 1 2; do
  bl "single auto" X=0
  for dp in 4 6; do bl "single TL=19 occ2 depth=$dp" ADL_BLOOM_TILE_LOG2=19 ADL_BLOOM_B_OCC=2 ADL_BLOOM_DEPTH=$dp; done
  BENCH_ARGS="--workload varlen" bl "varlen auto" X=0
  BENCH_ARGS="--workload varlen" bl "varlen TL=19 occ2 depth=4" ADL_BLOOM_TILE_LOG2=19 ADL_BLOOM_B_OCC=2 ADL_BLOOM_DEPTH=4
  BENCH_ARGS="--workload compaction --steps 10" bl "compaction auto" X=0
  for tl in 17 18 19; do
    for dp in 4 6; do
      BENCH_ARGS="--workload compaction --steps 10" bl "compaction TL=$tl occ2 depth=$dp" ADL_BLOOM_TILE_LOG2=$tl ADL_BLOOM_B_OCC=2 ADL_BLOOM_DEPTH=$dp
    done
  done
done
