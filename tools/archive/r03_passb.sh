#!/bin/bash
# tools/r03_passb.sh -- parity + full-size pins, then three headline and two
# compaction bench lines (pass B overlap check).
set -u
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pb_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pb_tests.log; [ $rc -ne 0 ] && exit $rc
AB="ADL_BLOOM_STAGES=2" REPS=3 timeout -k 10 400 bash tools/ab_env.sh || exit 1
AB="ADL_BLOOM_STAGES=2" REPS=2 BENCH_ARGS="--workload compaction" timeout -k 10 400 bash tools/ab_env.sh
