set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_primitives.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05o "new:QE_NOTHING=1" "prevmj:QE_LIB_PATH=$AB/libqe_r05n.so" || exit 1
echo all-done
