#!/bin/bash
# tools/r03_sweep.sh -- headline build at several key counts (pass A / pass B
# time per key: does a position round trip that fits the Infinity Cache run faster?)
set -u
cd "$(dirname "$0")/.."
for n in 2500000 5000000 10000000 20000000; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --keys $n --no-cpu-baseline --no-e2e > gpurun_out/sw_$n.json 2>/dev/null || exit 1
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]; print(sys.argv[2], d["value"], d["ms_per_step"], r["us_per_step"], r["positions_per_build"]["positions"], d["parity"])' gpurun_out/sw_$n.json $n
done
