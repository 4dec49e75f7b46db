#!/bin/bash
# tools/sweep_n.sh -- single-filter build at several key counts (per-key pass A/B cost vs size).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in ${SIZES:-1000000 2500000 5000000 10000000 20000000 40000000}; do
  out=$(timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 3 --keys $n --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} 2>/dev/null | grep '^{')
  rc=$?; [ $rc -ne 0 ] && { echo "n=$n rc=$rc"; exit $rc; }
  echo "$n :: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); n=d["config"]["keys_per_gpu"]; u=d["roofline"]["us_per_step"]; print(d["value"], {k: round(v/n*1e6,2) for k,v in u.items()}, "us/Mkey")')"
done | tee gpurun_out/sweep_n.log
