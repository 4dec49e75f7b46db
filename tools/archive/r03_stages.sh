timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rp_tests.log 2>&1; rc=$?; tail -2 gpurun_out/rp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 adlsm-tree_amd/bin/readpath_test --bench || exit 1
ADL_BLOOM_STAGES=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/st3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/st3_tests.log; [ $rc -ne 0 ] && exit $rc
AB="ADL_BLOOM_STAGES=2|ADL_BLOOM_STAGES=3" REPS=3 timeout -k 10 400 bash tools/ab_env.sh || exit 1
AB="ADL_BLOOM_STAGES=2|ADL_BLOOM_STAGES=3" REPS=2 BENCH_ARGS="--workload compaction" timeout -k 10 400 bash tools/ab_env.sh
