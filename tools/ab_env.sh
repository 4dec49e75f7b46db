#!/bin/bash
# tools/ab_env.sh -- interleaved A/B of bench.py under different env settings.
# usage: AB="ADL_BLOOM_CLAIM=0|ADL_BLOOM_CLAIM=1" REPS=3 bash tools/ab_env.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IFS='|' read -ra VARIANTS <<< "${AB}"
for rep in $(seq 1 ${REPS:-3}); do
  for v in "${VARIANTS[@]}"; do
    out=$(env $v timeout -k 10 300 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-e2e --no-sub-records --no-reader ${BENCH_ARGS:-} 2>/dev/null | grep '^{')
    rc=$?
    [ $rc -ne 0 ] && { echo "variant '$v' rc=$rc"; exit $rc; }
    echo "$v :: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])')"
  done
done | tee gpurun_out/ab.log
