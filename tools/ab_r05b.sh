set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_comm.py tests/test_gpu_fullsize.py tests/test_gpu_sort_cache.py > gpurun_out/r05b_tests.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh r05b_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "noprerank:QE_LIB_PATH=$AB/libqe_noprerank.so" "new:QE_NOTHING=1" || exit 1
bash tools/gpu_c4_ab.sh r05b "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "new:QE_NOTHING=1" || exit 1
echo all-done
