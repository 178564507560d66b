set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_local_ranks.py tests/test_gpu_comm.py > gpurun_out/r05g_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05g_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "tm1f:QE_LIB_PATH=$AB/libqe_p1tm1.so" "new:QE_NOTHING=1" "cs3:QE_CS_SINGLE=0" || exit 1
timeout -k 10 900 bash tools/round_end.sh r05g c3 || exit 1
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/r05g_c4_bench.json 2> gpurun_out/r05g_c4_bench.err || exit 1
timeout -k 10 400 bash tools/gpu_c4_timeline.sh r05g_c4tl plan || echo "c4 timeline failed rc=$?"
echo all-done
