#!/bin/bash
# tools/pb_variants.sh -- probe library variants on one box: the shape sweep
# entries in $PROBE_SHAPES and the configs[4] probe bench line, per library in
# $LIBS ("name:path name:path ...").
set -u
cd "$(dirname "$0")/.."
for l in $LIBS; do
  n=${l%%:*}; p=${l#*:}
  s=$(ADL_BLOOM_LIB=$p timeout -k 10 120 python3 tools/probe_shapes.py 2>/dev/null | python3 -c 'import json,sys; print(" ".join("F%d:%.3f" % (d["filters"], d["ms_median"]) for d in map(json.loads, sys.stdin) if d["sampled_answers_equal_oracle"]))') || exit 1
  b=$(ADL_BLOOM_LIB=$p timeout -k 10 200 python3 bench.py --workload probe --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | grep '^{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["parity"]["oracle"][:16])') || exit 1
  echo "$n :: shapes $s :: configs[4] $b"
done
