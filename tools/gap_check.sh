#!/bin/bash
# tools/gap_check.sh -- inter-kernel gaps of the headline build with pass A's
# position stores (EXP=2) or pass B's bitmap stores (EXP=8) switched off.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for e in ${EXPS:-0 2 8 10}; do
  ADL_BLOOM_EXP=$e timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/gap/e$e -o run --output-format csv -- \
    python3 tools/gap_probe.py > gpurun_out/gap_e$e.log 2>&1 || exit 1
  python3 - "$e" <<'PY'
import csv, glob, statistics as st, sys
f = glob.glob(f"gpurun_out/gap/e{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
bt = [k for k in ks if "bloom_bin" in k[2] or "bloom_tile" in k[2]][4:]
ab = [b[0] - a[1] for a, b in zip(bt, bt[1:]) if "tile" in b[2]]
ba = [b[0] - a[1] for a, b in zip(bt, bt[1:]) if "bin" in b[2]]
da = [k[1] - k[0] for k in bt if "bin" in k[2]]
db = [k[1] - k[0] for k in bt if "tile" in k[2]]
print(f"EXP={sys.argv[1]}: A {st.median(da)/1e3:.1f} us, gap A->B {st.median(ab)/1e3:.1f}, B {st.median(db)/1e3:.1f}, gap B->A {st.median(ba)/1e3:.1f}")
PY
done
