#!/bin/bash
# tools/r02_final2.sh -- round-2 evidence in one GPU call, after the build
# changes: PMC traffic passes (single, varlen) written into
# profiles/pmc_traffic.json first (bench.py reads it as roofline.traffic), then
# the GPU test suite, smoke(), the read-path latency bench, every bench
# workload with CPU baselines and a rocprofv3 kernel trace of the headline.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02b
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }
printf 'FETCH_SIZE\nWRITE_SIZE\nTCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum\n' > "$OUT/traffic_groups.txt"
for wl in single varlen; do
  step "pmc $wl"
  GROUPS_FILE=$OUT/traffic_groups.txt OUT=$OUT/pmc_$wl BENCH_ARGS="--workload $wl" bash tools/pmc.sh || exit 1
  ls $OUT/pmc_$wl/p1 > /dev/null || exit 1
  python3 tools/pmc_traffic.py "$OUT/pmc_$wl" profiles/pmc_traffic.json $wl > "$OUT/traffic_$wl.json" || exit 1
done
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
step readpath
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --bench > "$OUT/readpath_bench.json" 2> "$OUT/readpath_bench.err" || exit 1
step bench_all
bash tools/bench_all.sh || exit 1
cp gpurun_out/bench_all.jsonl "$OUT/bench_all.jsonl"
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit 1
step rocprof_varlen
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_varlen" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --workload varlen --no-cpu-baseline --no-e2e > "$OUT/prof_varlen_bench.json" 2> "$OUT/prof_varlen.err" || exit 1
exit 0
