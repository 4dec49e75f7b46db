#!/bin/bash
# tools/r03b_check.sh -- pb_tile diagnostics (wrong answers; timing only), then
# the full GPU test suite and smoke().
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03b_check
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=r03b_check/pbexp bash tools/r02_pbexp.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
