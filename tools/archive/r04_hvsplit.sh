#!/bin/bash
# tools/r04_hvsplit.sh -- var-len hashing pass: a run's longest key groups
# split between two waves by seed (ADL_BLOOM_HV_SPLIT = groups split), parity
# first (var-len GPU tests under each setting), then interleaved bench lines.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04h
mkdir -p $OUT
for sp in 1 2; do
  ADL_BLOOM_HV_SPLIT=$sp timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "varlen" > $OUT/parity_$sp.log 2>&1
  rc=$?; echo "split=$sp $(tail -1 $OUT/parity_$sp.log)"; [ $rc -eq 0 ] || exit $rc
done
bl() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --workload varlen --steps 20 --warmup 3 --no-e2e --no-cpu-baseline \
    2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']))"
}
for rep in 1 2 3; do
  for sp in 0 1 2; do bl "split=$sp" ADL_BLOOM_HV_SPLIT=$sp; done
done
