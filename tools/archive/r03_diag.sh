#!/bin/bash
# tools/r03_diag.sh -- pass-A/B phase stamps under diagnostics switches
# (ADL_BLOOM_EXP: 1 no hash, 2 no position stores, 32 no reduction; wrong
# bitmaps, stamps build only) and ADL_BLOOM_HOT.  Usage: CASES="0:1 1:1" bash tools/r03_diag.sh
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r03_diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CASES:-0:0 0:1 1:1 32:1 33:1 2:1 35:1}; do
  e=${c%%:*}; h=${c##*:}
  echo "=== EXP=$e HOT=$h"
  ADL_BLOOM_EXP=$e ADL_BLOOM_HOT=$h timeout -k 10 120 python3 tools/stamps.py > "$OUT/stamps_${e}_${h}.txt" 2>&1 || { cat "$OUT/stamps_${e}_${h}.txt"; exit 1; }
  cat "$OUT/stamps_${e}_${h}.txt"
done
