#!/bin/bash
# tools/r05_lds_ab.sh -- round 5: the LDS-conflict ceiling of pass A (the
# diagnostics build's conflict-free sort, ADL_BLOOM_EXP=64, against the same
# build's real sort, with and without the hash dedup), then the read-path
# tails and Gets-beside-builds runs of readpath_test.  TAG names gpurun_out/.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --tails 220000 > "$OUT/tails.json" 2> "$OUT/tails.err" || exit 1
cat "$OUT/tails.json"
timeout -k 10 200 adlsm-tree_amd/bin/readpath_test --coexist 40 > "$OUT/coexist.json" 2> "$OUT/coexist.err" || exit 1
cat "$OUT/coexist.json"
export ADL_BLOOM_LIB=adlsm-tree_amd/lib_stamps/libadlbloom.so
AB="ADL_BLOOM_EXP=0|ADL_BLOOM_EXP=64|ADL_BLOOM_EXP=0 ADL_BLOOM_HASH_DEDUP=0|ADL_BLOOM_EXP=64 ADL_BLOOM_HASH_DEDUP=0" \
  REPS=3 STEPS=30 bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/lds_ab.log"
