set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/srv_inline; mkdir -p $OUT
timeout -k 10 150 python -u -m pytest tests/test_gpu_readpath.py -q -x --timeout 60 --timeout-method thread -p no:cacheprovider > $OUT/pytest_readpath.log 2>&1
rc=$?; tail -3 $OUT/pytest_readpath.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export LD_LIBRARY_PATH=$PWD/abl/srvbase; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --bench > $OUT/bench_$v$rep.json 2>/dev/null || exit 1
    timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --tails 100000 > $OUT/tails_$v$rep.json 2>/dev/null || exit 1
    echo "$v$rep bench $(head -c 120 $OUT/bench_$v$rep.json)"
    echo "$v$rep tails $(head -c 200 $OUT/tails_$v$rep.json)"
  done
done
