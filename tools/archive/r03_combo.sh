#!/bin/bash
# tools/r03_combo.sh -- GPU tests (var-len parity, probe batch, full-size pins),
# then A/Bs: hashing-pass staging bytes (varlen) and the probe's K2 scan.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_combo}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py \
  -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
AB="ADL_PB_OLDSCAN=1|ADL_PB_NEWSCAN=1" REPS=2 STEPS=5 BENCH_ARGS="--workload probe" timeout -k 10 600 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab_probe_scan.log"
AB="ADL_BLOOM_HV_STAGE=48|ADL_BLOOM_HV_STAGE=40|ADL_BLOOM_HV_STAGE=36" REPS=2 STEPS=30 BENCH_ARGS="--workload varlen" timeout -k 10 600 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/ab_hv_stage.log"
