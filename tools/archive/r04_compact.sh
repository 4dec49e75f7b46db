#!/bin/bash
# tools/r04_compact.sh -- pass A live-key compaction (collapsed keys stamped,
# live keys ranked across the workgroup and staged densely) against the
# round-3 pass A: parity first, then interleaved bench lines and one PMC pass
# (SQ_INSTS_LDS) per variant.  Each step time-limited; a failed step ends it.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04c
mkdir -p $OUT
bl() {  # one bench line: label, env..., args
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-compaction-strong --no-e2e --no-cpu-baseline \
    ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'] if isinstance(d['parity'], str) else d['parity'].get('oracle'), json.dumps(r['us_per_step']), (r.get('positions_per_build') or {}).get('positions'))"
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "build or sstable" \
  > $OUT/parity.log 2>&1; rc=$?; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  bl "r3   " ADL_BLOOM_HOT=0
  bl "hot  " ADL_BLOOM_HOT=1 ADL_BLOOM_COMPACT=0
  bl "cmp  " ADL_BLOOM_HOT=1 ADL_BLOOM_COMPACT=1
done
for rep in 1 2; do
  BENCH_ARGS="--workload compaction --steps 10" bl "compaction r3 " ADL_BLOOM_HOT=0
  BENCH_ARGS="--workload compaction --steps 10" bl "compaction cmp" ADL_BLOOM_HOT=1
done
printf 'SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE\n' > $OUT/lds_group.txt
for v in 0 1; do
  ADL_BLOOM_HOT=$v GROUPS_FILE=$OUT/lds_group.txt OUT=$OUT/lds_hot$v bash tools/pmc.sh || exit 1
done
