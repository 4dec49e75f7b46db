#!/bin/bash
# tools/r03_varlen.sh -- var-len build: parity (parity tests with var-len keys,
# the configs[2] full-size pin), then the varlen bench line and a rocprofv3
# kernel trace of it.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03_varlen${1:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q \
  -k "var or Var or full" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --workload varlen --no-cpu-baseline --no-e2e > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["roofline"]["frac"], d["parity"])' "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 3 --workload varlen --no-cpu-baseline --no-e2e > "$OUT/prof.json" 2> "$OUT/prof.err" || exit 1
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -8 {} \;
