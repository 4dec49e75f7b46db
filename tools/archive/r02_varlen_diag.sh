#!/bin/bash
# tools/r02_varlen_diag.sh -- var-len pass A evidence: phase stamps (diagnostics
# build) and PMC passes over bench.py --workload varlen.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r02/varlen
mkdir -p "$OUT"
export TMPDIR=/tmp
WORKLOAD=varlen timeout -k 10 300 python3 tools/stamps.py > "$OUT/stamps.txt" 2>&1; echo "stamps rc=$?"; cat "$OUT/stamps.txt" | grep -v amdgpu.ids
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    python3 bench.py --workload varlen --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done < tools/pmc_groups.txt
exit 0
