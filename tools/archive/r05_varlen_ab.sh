#!/bin/bash
# tools/r05_varlen_ab.sh -- the var-len long-key split on the GPU: its parity
# tests and the configs[2] pin, then the var-len bench under ADL_BLOOM_HV_LONG
# = 0 (off) and 128, interleaved, with rocprofv3 kernel stats of one run each.
# TAG names gpurun_out/.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:?set TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "varlen" -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_varlen.log" 2>&1
rc=$?; tail -n 5 "$OUT/pytest_varlen.log"; [ $rc -ne 0 ] && exit $rc
AB="ADL_BLOOM_HV_LONG=0|ADL_BLOOM_HV_LONG=128" REPS=3 STEPS=20 BENCH_ARGS="--workload varlen" bash tools/ab_env.sh || exit 1
cp gpurun_out/ab.log "$OUT/varlen_ab.log"
for v in 0 128; do
  ADL_BLOOM_HV_LONG=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/s$v" -o run --output-format csv -- \
    python3 bench.py --workload varlen --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > /dev/null 2>&1 || exit 1
  python3 - "$OUT/s$v" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    row = []
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("hash_var", "hash_long", "bloom_bin", "bloom_tile"):
            if k in n:
                row.append("%s=%.1f" % (k, float(r["AverageNs"]) / 1e3))
    print("HV_LONG=%s: %s" % (sys.argv[2], " ".join(row)))
PY
done
