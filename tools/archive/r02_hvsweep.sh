#!/bin/bash
# tools/r02_hvsweep.sh -- var-len bench over hashing-run sizes (ADL_BLOOM_HV_KEYS)
# and the fused pass A (ADL_BLOOM_VAR_HASH=0), after a short parity check.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/hvsweep
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "varlen or zipf" > "$OUT/pytest.log" 2>&1; rc=$?; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
# entries lib:var_hash:hv_keys, lib = cur (adlsm-tree_amd/lib) or ab (adlsm-tree_amd/lib_ab, an A/B build)
for cfg in ${CFGS:-cur:1:512 ab:1:512 cur:1:512 ab:1:512 cur:0:512}; do
  IFS=: read -r lib vh hk <<< "$cfg"
  L=""; [ "$lib" = ab ] && L="$PWD/adlsm-tree_amd/lib_ab/libadlbloom.so"
  ADL_BLOOM_LIB=$L ADL_BLOOM_VAR_HASH=$vh ADL_BLOOM_HV_KEYS=$hk timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 \
    --workload varlen --no-cpu-baseline --no-e2e > "$OUT/bench_${lib}_${vh}_${hk}.log" 2>&1 || exit 1
  echo -n "$lib VAR_HASH=$vh HV_KEYS=$hk: "
  grep '^{' "$OUT/bench_${lib}_${vh}_${hk}.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_step"], d["parity"])'
done
exit 0
