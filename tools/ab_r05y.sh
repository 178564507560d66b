# r05y: pass 1 / pass 2 / the local sort with every kernel argument fetched in one scalar round before the first load -- GPU tests, C3 and C4 new/prev
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/r05y_tests.log 2>&1 || exit 1
REPS=3 timeout -k 10 700 bash tools/gpu_lib_ab.sh r05y_c3 "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05y "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
echo all-done
