#!/bin/bash
# tools/r05_probe_check.sh -- a probe change on the GPU: the binned-probe tests
# (shape sweep, unaligned output, the full 100M-query configs[4] pin), then the
# probe bench line and its rocprofv3 kernel stats.  TAG names gpurun_out/.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py -k "probe" -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_probe.log" 2>&1
rc=$?; tail -n 5 "$OUT/pytest_probe.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --workload probe --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > "$OUT/bench_probe.json" 2> "$OUT/bench_probe.err" || exit 1
cut -c1-420 "$OUT/bench_probe.json"
python3 - "$OUT/stats" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    row = []
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "pb_" in n:
            row.append("%s=%.0f" % (n[n.index("pb_"):].split("(")[0].split("<")[0], float(r["AverageNs"]) / 1e3))
    print(" ".join(row))
PY
