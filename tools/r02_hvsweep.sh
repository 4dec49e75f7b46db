#!/bin/bash
# tools/r02_hvsweep.sh -- var-len bench over hashing-run sizes (ADL_BLOOM_HV_KEYS)
# and the fused pass A (ADL_BLOOM_VAR_HASH=0), after a short parity check.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/hvsweep
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "varlen or zipf" > "$OUT/pytest.log" 2>&1; rc=$?; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-1:512 1:1024 1:2048 0:1024}; do
  set -- ${cfg/:/ }
  ADL_BLOOM_VAR_HASH=$1 ADL_BLOOM_HV_KEYS=$2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload varlen \
    --no-cpu-baseline --no-e2e > "$OUT/bench_$1_$2.log" 2>&1 || exit 1
  echo -n "VAR_HASH=$1 HV_KEYS=$2: "
  grep '^{' "$OUT/bench_$1_$2.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])'
done
exit 0
