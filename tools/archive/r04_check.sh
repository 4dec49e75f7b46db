#!/bin/bash
# tools/r04_check.sh -- round-4 bring-up in one GPU call: bucketed-build stamps,
# correctness shapes (u32 and 24-bit entries), headline A/B over the build
# variants, the probe tests and the K3 run-store A/B.  Each step time-limited;
# a failed correctness step ends the call.
set -u
cd "$(dirname "$0")/.."
bl() {  # one bench line: label, env..., args
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-compaction-strong --no-e2e --no-cpu-baseline \
    ${BENCH_ARGS:-} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$label', d['value'], d['ms_per_step'], d['parity'] if isinstance(d['parity'], str) else d['parity'].get('oracle'), json.dumps(r['us_per_step']), (r.get('positions_per_build') or {}).get('positions'))"
}
timeout -k 10 120 python3 tools/stamps.py 2>&1 | grep -v amdgpu.ids | head -20
timeout -k 10 200 python3 tools/dbg_bk.py 2>&1 | grep -v amdgpu.ids || exit 1
ADL_BLOOM_BK_P3=1 timeout -k 10 200 python3 tools/dbg_bk.py 2>&1 | grep -v amdgpu.ids || exit 1
for rep in 1 2; do
  bl "bk-u32" ADL_BLOOM_BK_P3=0
  bl "bk-p3 " ADL_BLOOM_BK_P3=1
  bl "old   " ADL_BLOOM_BK=0
done
BENCH_ARGS="--keys 2500000" bl "bk-u32 2.5M" ADL_BLOOM_BK_P3=0
BENCH_ARGS="--keys 2500000" bl "bk-p3 2.5M" ADL_BLOOM_BK_P3=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_probe_batch.py 2>&1 | tail -2
for fl in 0 1; do BENCH_ARGS="--workload probe --steps 10" bl "probe flat=$fl" ADL_PB_FLAT=$fl; done
