#!/bin/bash
# tools/pmc.sh -- rocprofv3 PMC passes over a short bench run, one counter
# group per pass (never combined with sys/runtime traces).  A pass that fails
# with an ordinary error (e.g. an unknown counter) is skipped; a signal or
# timeout ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=(python3 bench.py --steps ${PMC_STEPS:-4} --warmup 1 --no-cpu-baseline --no-e2e --no-compaction-strong --no-sub-records --no-reader ${BENCH_ARGS:-})
[ "${LIST:-0}" = 1 ] && { timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"; }
i=0
while IFS= read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "=== pass $i: $group"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$OUT/p$i" -o run --output-format csv -- "${CMD[@]}" \
    > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done < "${GROUPS_FILE:-tools/pmc_groups.txt}"
exit 0
