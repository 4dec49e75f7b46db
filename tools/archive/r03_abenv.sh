#!/bin/bash
# tools/r03_abenv.sh -- parity + full-size GPU tests (working tree), then an
# interleaved A/B over environment settings (AB="X=0|X=1").
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_abenv}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_full_size.py} -x -q -rf \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
AB="$AB" REPS=${REPS:-3} STEPS=30 timeout -k 10 900 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab.log"
