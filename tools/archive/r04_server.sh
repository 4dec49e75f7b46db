#!/bin/bash
# tools/r04_server.sh -- the resident probe server: its GPU tests, then the
# read-path latency bench with the server and without it (launch per Get).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r04s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_readpath.py \
  -k "probe_server or completion_fault or small_batch" > $OUT/server_tests.log 2>&1; rc=$?
tail -12 $OUT/server_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  ADL_BLOOM_PROBE_SERVER=$v timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --bench > $OUT/readpath_server$v.json 2>&1 || exit 1
  echo "server=$v $(cat $OUT/readpath_server$v.json)"
done
