#!/bin/bash
# tools/r04_groups.sh -- configs[3] compaction (256 tables x 1M keys) in groups
# of G tables per launch pair (ADL_BLOOM_GROUP_KEYS = G x 1M keys), so each
# group's positions (24 B per key) stay inside the 256 MiB Infinity Cache,
# against one launch pair for all 256 tables; interleaved reps.
set -u
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for g in 0 8 10 16 32; do
    if [ $g = 0 ]; then E=(); else E=(ADL_BLOOM_GROUP_KEYS=$((g * 1000000))); fi
    env "${E[@]}" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --workload compaction --no-e2e \
      --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('group $g', d['value'], d['ms_per_step'], d['parity'], json.dumps(r['us_per_step']), r['launch_pairs_per_build'])"
  done
done
