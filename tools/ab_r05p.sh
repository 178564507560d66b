set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
QE_LIB_PATH=$AB/libqe_hwrows.so timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p_hwrows_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05p_c3 "new:QE_NOTHING=1" "hwrows:QE_LIB_PATH=$AB/libqe_hwrows.so" "tpg512:QE_LIB_PATH=$AB/libqe_tpg512.so" || exit 1
echo all-done
