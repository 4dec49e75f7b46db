#!/bin/bash
# tools/r03_split.sh -- the two-round binned probe: probe parity tests (small
# shapes + the 100 M-query pin) under each ADL_PB_SPLIT, then an interleaved
# bench A/B over the splits.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_split}
mkdir -p "$OUT"
export TMPDIR=/tmp
for sp in ${SPLITS:-1 2}; do
  ADL_PB_SPLIT=$sp timeout -k 10 400 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py \
    -x -q -k probe --timeout 300 --timeout-method thread > "$OUT/pytest_split$sp.log" 2>&1
  rc=$?; echo "split $sp pytest rc=$rc"; tail -n 2 "$OUT/pytest_split$sp.log"; [ $rc -ne 0 ] && exit $rc
done
AB="${AB:-ADL_PB_SPLIT=0|ADL_PB_SPLIT=1|ADL_PB_SPLIT=2}" REPS=${REPS:-3} STEPS=20 \
  BENCH_ARGS="--workload probe" timeout -k 10 900 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab.log"
