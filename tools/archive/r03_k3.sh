#!/bin/bash
# tools/r03_k3.sh -- the persistent K3 (ADL_PB_SCATTER_P=1): probe tests under
# it, then an interleaved A/B against the one-block-per-workgroup K3.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03_k3
mkdir -p "$OUT"
export TMPDIR=/tmp
ADL_PB_SCATTER_P=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py -k probe \
  -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
AB="ADL_PB_SCATTER_P=0|ADL_PB_SCATTER_P=1" REPS=3 STEPS=5 BENCH_ARGS="--workload probe" timeout -k 10 600 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab.log"
