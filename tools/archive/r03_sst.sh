#!/bin/bash
# tools/r03_sst.sh -- SSTable tests (plain and overlapped Final) and the
# compaction-shaped flush benchmark: t tables, Final per table vs filling
# table t+1 while table t's filter builds.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03_sst
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k sstable -x -q -rf --timeout 200 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for nt in "100000 8" "1000000 4"; do
  timeout -k 10 300 adlsm-tree_amd/bin/sstable_test pipebench $nt | tee -a "$OUT/pipebench.jsonl" || exit 1
done
