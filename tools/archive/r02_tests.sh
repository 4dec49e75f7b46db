#!/bin/bash
# tools/r02_tests.sh -- GPU parity suite + the read-path latency bench.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "=== pytest ($(date +%T))"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 30 "$OUT/pytest_gpu.log"
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
echo "=== readpath bench ($(date +%T))"
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --bench > "$OUT/readpath_bench.json" 2> "$OUT/readpath_bench.err"
rc2=$?; echo "readpath rc=$rc2"; cat "$OUT/readpath_bench.json"; tail -3 "$OUT/readpath_bench.err"
exit $rc
