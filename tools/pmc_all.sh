#!/bin/bash
# tools/pmc_all.sh -- PMC passes per workload into profiles/pmc_traffic.json:
# FETCH_SIZE, WRITE_SIZE (traffic; tools/pmc_traffic.py), the integer-issue
# group (tools/pmc_alu.py) and the LDS group (array / bank-conflict cycles,
# tools/pmc_lds.py).  Each pass its own rocprofv3 run (tools/pmc.sh).
# usage: bash tools/pmc_all.sh OUTDIR workload...
set -u
cd "$(dirname "$0")/.."
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
printf 'FETCH_SIZE\nWRITE_SIZE\nTCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum\n' > "$OUT/traffic_groups.txt"
printf 'SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE\n' > "$OUT/alu_groups.txt"
printf 'SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE\n' \
  > "$OUT/lds_groups.txt"
for wl in "$@"; do
  echo "=== pmc $wl ($(date +%T))"
  GROUPS_FILE=$OUT/traffic_groups.txt OUT=$OUT/pmc_$wl BENCH_ARGS="--workload $wl" bash tools/pmc.sh || exit 1
  python3 tools/pmc_traffic.py "$OUT/pmc_$wl" profiles/pmc_traffic.json $wl > "$OUT/traffic_$wl.json" || exit 1
  if [ "$wl" != probe ]; then
    GROUPS_FILE=$OUT/alu_groups.txt OUT=$OUT/alu_$wl BENCH_ARGS="--workload $wl" bash tools/pmc.sh || exit 1
    python3 tools/pmc_alu.py "$OUT/alu_$wl" profiles/pmc_traffic.json $wl > "$OUT/alu_$wl.json" || exit 1
    GROUPS_FILE=$OUT/lds_groups.txt OUT=$OUT/lds_$wl BENCH_ARGS="--workload $wl" bash tools/pmc.sh || exit 1
    python3 tools/pmc_lds.py "$OUT/lds_$wl" profiles/pmc_traffic.json $wl > "$OUT/lds_$wl.json" || exit 1
  fi
done
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
