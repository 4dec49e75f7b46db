#!/bin/bash
# tools/r02_pmc_probe.sh -- PMC traffic passes over the probe workload (one counter group per pass).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02/pmc_probe_b
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    python3 bench.py --workload probe --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
