#!/bin/bash
# tools/bench_all.sh -- every bench workload on one GPU, each with its own time
# limit; the JSON lines go to gpurun_out/bench_all.jsonl.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/bench_all.jsonl
for wl in ${WORKLOADS:-single varlen compaction probe}; do
  timeout -k 10 600 python3 bench.py --steps ${STEPS:-20} --warmup 3 --workload $wl ${BENCH_ARGS:-} \
    > gpurun_out/bench_$wl.log 2>&1
  rc=$?
  echo "=== $wl rc=$rc"
  grep '^{' gpurun_out/bench_$wl.log >> gpurun_out/bench_all.jsonl
  grep '^{' gpurun_out/bench_$wl.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", d["roofline"]["us_per_step"], d["roofline"]["frac"], d["parity"])' || tail -5 gpurun_out/bench_$wl.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
