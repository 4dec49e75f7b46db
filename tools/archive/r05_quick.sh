set -u
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2 3; do
  ADL_BLOOM_SERVER_LIFE_US=2000 timeout -k 5 20 adlsm-tree_amd/bin/readpath_test --tails 20000 > $OUT/tails_$i.json 2> $OUT/tails_$i.err
  rc=$?; echo "run $i rc=$rc"; [ $rc -ne 0 ] && { tail -4 $OUT/tails_$i.err; exit 1; }
done
cat $OUT/tails_3.json
timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --tails 200000 > $OUT/tails.json 2> $OUT/tails.err || exit 1
cat $OUT/tails.json
timeout -k 10 200 adlsm-tree_amd/bin/readpath_test --coexist 20 > $OUT/coexist.json 2> $OUT/coexist.err || exit 1
cat $OUT/coexist.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_readpath.py -q -x --timeout 100 --timeout-method thread -p no:cacheprovider > $OUT/pytest_readpath.log 2>&1; rc=$?
tail -3 $OUT/pytest_readpath.log; exit $rc
