#!/bin/bash
# tools/r05_check.sh -- round 5 check call: the GPU suite, smoke(), a headline
# bench line, the read-path coexistence run (Gets beside builds) and the
# probe-server tail run.  TAG names the gpurun_out/ directory.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }
step pytest
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 12 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
step bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-e2e --no-compaction-strong --no-cpu-baseline \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cut -c1-400 "$OUT/bench.json"
step coexist
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --coexist 20 > "$OUT/coexist.json" 2> "$OUT/coexist.err" || exit 1
cat "$OUT/coexist.json"
step tails
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --tails 200000 > "$OUT/tails.json" 2> "$OUT/tails.err" || exit 1
cat "$OUT/tails.json"
exit $rc
