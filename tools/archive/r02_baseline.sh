#!/bin/bash
# tools/r02_baseline.sh -- one gpurun session: smoke, the GPU parity suite, and
# the probe workload's evidence (bench line, rocprofv3 kernel trace, PMC
# traffic passes).  Every GPU step has its own time limit; a fault / abort /
# timeout ends the script before anything else touches the GPU.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  return $rc
}
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }

step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
  rc=$?; fatal $rc && exit $rc
fi
step bench_probe 600 python bench.py --workload probe --steps 10 --warmup 2 --no-cpu-baseline || exit $?
step rocprof_probe 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o run --output-format csv -- \
  python3 bench.py --workload probe --steps 10 --warmup 2 --no-cpu-baseline || exit $?
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  step pmc_probe_$i 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc_probe/p$i" -o run --output-format csv -- \
    python3 bench.py --workload probe --steps 2 --warmup 1 --no-cpu-baseline || exit $?
done
exit 0
