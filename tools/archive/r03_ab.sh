#!/bin/bash
# tools/r03_ab.sh -- parity + full-size GPU tests of the working tree, then an
# interleaved A/B of the headline against the base library (abl/base).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_full_size.py} -x -q -rf \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
LIBS="${LIBS:-abl/base/libadlbloom.so|adlsm-tree_amd/lib/libadlbloom.so}" REPS=${REPS:-3} STEPS=30 timeout -k 10 600 bash tools/ab_lib.sh || exit 1
cp gpurun_out/ab_lib.log "$OUT/ab_lib.log"
