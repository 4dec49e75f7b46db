#!/bin/bash
# tools/r04_ab_nox.sh -- pass B: lanes past a segment read its first word
# (abl/nox) vs the next segment's words (abl/base); interleaved, three workloads.
set -u
cd "$(dirname "$0")/.."
for rep in 1 2 3; do
  for lib in base nox; do
    for wl in single varlen; do
      ADL_BLOOM_LIB=abl/$lib/libadlbloom.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload $wl \
        --no-compaction-strong --no-e2e --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib $wl', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']))"
    done
  done
done
