#!/bin/bash
# tools/r06_check.sh -- round 6 check call, steps chosen by environment:
#   PYTEST="paths"  GPU tests first (-x, a per-test time limit)
#   BENCH=1         the default bench line (headline, compaction_strong,
#                   headline_with_reader, probe and varlen sub-records)
#   AB_PROBE=n      n interleaved reps of bench.py --workload probe over
#                   abl/base/libadlbloom.so and the current library
#   COEXIST="2 0 1" reads-beside-builds (readpath_test --coexist) under the
#                   build-queue policies ADL_BLOOM_BUILD_QUEUES=v (0 static,
#                   1 while a server exists = round 5, 2 while a server kernel
#                   is resident = default); PASSES=1: pass A only
#   TAILS=n         readpath_test --tails n (the server's phase stamps)
#   PROF_PROBE=1    rocprofv3 kernel stats of bench.py --workload probe on
#                   abl/base/libadlbloom.so and on the current library
#   E2E_PARTS=1     tools/e2e_parts.py (a host-to-host build's parts)
#   INV_AB=1        coexist with ADL_BLOOM_SERVER_INVALIDATE=1 (the server
#                   invalidates its caches at every request, round 5) and 0
#   DEBUG=1         the coexist runs with ADL_BLOOM_DEBUG=1 (slow Gets logged
#                   with the server kernel's phase stamps)
# Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2> "$OUT/$name.err"
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$OUT/$name.log" "$OUT/$name.err"
  return $rc
}
if [ -n "${PYTEST:-}" ]; then
  step pytest 900 python -u -m pytest $PYTEST -m gpu -x -q --timeout 300 --timeout-method thread -rf || exit $?
fi
if [ "${BENCH:-0}" = 1 ]; then
  step bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
fi
if [ -n "${AB_PROBE:-}" ]; then
  for rep in $(seq 1 $AB_PROBE); do
    for lib in abl/base/libadlbloom.so adlsm-tree_amd/lib/libadlbloom.so; do
      n=$(basename $(dirname $lib))
      ADL_BLOOM_LIB=$lib step ab_probe_${n}_$rep 300 python bench.py --workload probe --steps 20 --warmup 3 \
        --no-cpu-baseline --no-e2e || exit $?
    done
  done
  grep -h '^{' "$OUT"/ab_probe_*.log | python3 -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"]["oracle"])' | tee "$OUT/ab_probe.txt"
fi
if [ "${PROF_PROBE:-0}" = 1 ]; then
  for lib in abl/base/libadlbloom.so adlsm-tree_amd/lib/libadlbloom.so; do
    n=$(basename $(dirname $lib))
    ADL_BLOOM_LIB=$lib step prof_probe_$n 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe_$n" -o run \
      --output-format csv -- python3 bench.py --workload probe --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
      || exit $?
    python3 tools/kstats_pb.py "$OUT/prof_probe_$n" | tee -a "$OUT/prof_probe.txt"
  done
fi
for v in ${COEXIST:-}; do
  ADL_BLOOM_DEBUG=${DEBUG:-0} ADL_BLOOM_BUILD_QUEUES=$v step coexist_q$v 300 adlsm-tree_amd/bin/readpath_test --coexist ${REPS:-20} || exit $?
done
if [ "${INV_AB:-0}" = 1 ]; then
  for inv in 1 0; do
    ADL_BLOOM_SERVER_INVALIDATE=$inv step coexist_inv$inv 300 adlsm-tree_amd/bin/readpath_test --coexist ${REPS:-20} \
      || exit $?
  done
fi
if [ -n "${PASSES:-}" ]; then
  ADL_BLOOM_BUILD_QUEUES=2 ADL_BLOOM_BUILD_QUEUE_PASSES=$PASSES step coexist_q2_p$PASSES 300 \
    adlsm-tree_amd/bin/readpath_test --coexist ${REPS:-20} || exit $?
fi
if [ "${E2E_PARTS:-0}" = 1 ]; then
  step e2e_parts 300 python3 tools/e2e_parts.py || exit $?
fi
if [ -n "${TAILS:-}" ]; then
  step tails 300 adlsm-tree_amd/bin/readpath_test --tails $TAILS || exit $?
fi
exit 0
