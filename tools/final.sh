#!/bin/bash
# tools/final.sh -- one round's evidence in one GPU call: PMC passes (traffic +
# integer issue) written into profiles/pmc_traffic.json first (bench.py reads
# them), the GPU test suite, smoke(), the read-path latency bench, Gets beside
# builds (readpath_test --coexist) and the server's tails, every bench
# workload with CPU baselines, rocprofv3 kernel traces of the headline,
# var-len and probe runs, and the driver's default bench line.
# SKIP_PMC=1 / PMC_ONLY=1 split it over two calls (PMC_WORKLOADS= to narrow).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG, e.g. TAG=r04a}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "=== $1 ($(date +%T))"; }
if [ "${SKIP_PMC:-0}" != 1 ]; then
  step pmc
  bash tools/pmc_all.sh "$OUT/pmc" ${PMC_WORKLOADS:-single varlen compaction probe} > "$OUT/pmc.log" 2>&1 || { tail -5 "$OUT/pmc.log"; exit 1; }
  if [ "${PMC_ONLY:-0}" = 1 ]; then
    step bench_default
    timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit 1
    tail -c 400 "$OUT/bench_default.json"
    exit 0
  fi
fi
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit 1
tail -n 1 "$OUT/smoke.log"
step readpath
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --bench > "$OUT/readpath_bench.json" 2> "$OUT/readpath_bench.err" || exit 1
step readpath_coexist_tails
timeout -k 10 300 adlsm-tree_amd/bin/readpath_test --coexist 40 > "$OUT/coexist.json" 2> "$OUT/coexist.err" || exit 1
ADL_BLOOM_SERVER_LIFE_US=20000 timeout -k 10 200 adlsm-tree_amd/bin/readpath_test --tails 220000 > "$OUT/tails.json" 2> "$OUT/tails.err" || exit 1
step sstable_pipebench
for nt in "100000 8" "1000000 4"; do
  timeout -k 10 300 adlsm-tree_amd/bin/sstable_test pipebench $nt >> "$OUT/sstable_pipebench.jsonl" || exit 1
done
step bench_all
bash tools/bench_all.sh || exit 1
cp gpurun_out/bench_all.jsonl "$OUT/bench_all.jsonl"
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-compaction-strong --no-sub-records --no-reader > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit 1
step rocprof_varlen
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_varlen" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --workload varlen --no-cpu-baseline --no-e2e > "$OUT/prof_varlen_bench.json" 2> "$OUT/prof_varlen.err" || exit 1
step rocprof_probe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --workload probe --no-cpu-baseline --no-e2e > "$OUT/prof_probe_bench.json" 2> "$OUT/prof_probe.err" || exit 1
step bench_default
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit 1
tail -c 400 "$OUT/bench_default.json"
exit 0
