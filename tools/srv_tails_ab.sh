#!/bin/bash
# tools/srv_tails_ab.sh -- the resident probe server's single-key latency
# (readpath_test --tails) over library builds, interleaved:
# LIBDIRS="abl/srv8 adlsm-tree_amd/lib" REPS=2 CALLS=100000 bash tools/srv_tails_ab.sh
# (a directory holding libadlbloom.so goes first on LD_LIBRARY_PATH).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-srv_tails_ab}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for d in ${LIBDIRS}; do
    n=$(echo $d | tr '/' '_')
    LD_LIBRARY_PATH=$PWD/$d timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --tails ${CALLS:-100000} \
      > $OUT/tails_${n}_$rep.json 2> $OUT/tails_${n}_$rep.err || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$OUT/tails_${n}_$rep.json').read().strip().splitlines()[-1])
s=d['single_key_us']; p=d['server_phases_us']
print('$d rep $rep: p50 %.2f p99 %.2f max %.1f | kernel: loads %.2f staged %.2f hashed %.2f read %.2f answered %.2f host %.2f' % (s['p50'], s['p99'], s['max'], p['poll_loads_back'], p['slot_staged'], p['hashed'], p['bits_read'], p['answer_stored'], p['host_per_request']))" | tee -a $OUT/summary.txt
  done
done
