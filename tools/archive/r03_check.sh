#!/bin/bash
# tools/r03_check.sh -- full GPU test suite, then the headline and compaction
# bench lines and the PCIe duplex probe.  Usage: bash tools/r03_check.sh [tag]
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03_${1:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 6 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for wl in ${WORKLOADS:-single compaction}; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || exit 1
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d.get("launch_pairs_per_build"), d["parity"], d.get("e2e"))' "$OUT/bench_$wl.json" $wl
done
timeout -k 10 120 python3 tools/pcie_duplex.py > "$OUT/pcie.json" 2>&1; cat "$OUT/pcie.json"
