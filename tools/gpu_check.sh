#!/bin/bash
# tools/gpu_check.sh -- one gpurun session: smoke, GPU parity tests, a short
# bench and a rocprofv3 kernel-trace summary.  Each GPU step has its own time
# limit; a fault / abort / timeout (exit >= 2 other than pytest's 1) ends the
# script before anything else touches the GPU.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  return $rc
}

ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu ${PYTEST_SECS:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}
rc=$?; ok_or_testfail $rc || exit $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
step bench 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} || exit $?
cat "$OUT/bench.log" | grep '^{' > "$OUT/bench.json" || true
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e || exit $?
find "$OUT/prof" -name "*kernel_stats.csv" | head -5
exit 0
