#!/bin/bash
# tools/r03_hot.sh -- collapsed-key stamping: its tests, the parity and
# full-size GPU suites, then an interleaved A/B of ADL_BLOOM_HOT (pair table on/off).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_hot}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hot_keys.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q -rf \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
AB="ADL_BLOOM_HOT=0|ADL_BLOOM_HOT=1|ADL_BLOOM_HOT=1 ADL_BLOOM_HASH_DEDUP=0" REPS=3 STEPS=30 timeout -k 10 600 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab.log"
