#!/bin/bash
# tools/r03_probe.sh -- probe parity (probe tests, configs[4] pin) and two probe bench lines
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest tests/test_gpu_probe_batch.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pr_tests.log 2>&1; rc=$?; tail -2 gpurun_out/pr_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --workload probe --no-cpu-baseline --no-e2e > gpurun_out/pr_$i.json 2>/dev/null || exit 1
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["parity"]["oracle"])' gpurun_out/pr_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pr_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --workload probe --no-cpu-baseline --no-e2e > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/pr_prof/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'pb_' in r['Name']: print(r['Name'].split('(')[0][-30:], round(float(r['AverageNs'])/1e3,1))
PY
