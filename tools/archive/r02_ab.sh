#!/bin/bash
# tools/r02_ab.sh -- interleaved A/B of one environment knob on a bench
# workload, after the parity tests with the knob on.
#   KNOB=ADL_BLOOM_HASH_DEDUP VALS="0 1 0 1" WL=single bash tools/r02_ab.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/ab
mkdir -p "$OUT"
KNOB=${KNOB:?} ; WL=${WL:-single}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} \
    > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest: $(tail -n 1 $OUT/pytest.log)"; [ $rc -ne 0 ] && exit $rc
fi
for v in ${VALS:-0 1 0 1}; do
  tag=$(basename "$(dirname "$v")")_$(basename "$v")
  for wl in $WL; do
    env $KNOB=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload $wl --no-cpu-baseline --no-e2e \
      > "$OUT/bench_${wl}_$tag.log" 2>&1 || exit 1
    echo -n "$wl $KNOB=$v: "
    grep '^{' "$OUT/bench_${wl}_$tag.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])'
  done
done
exit 0
