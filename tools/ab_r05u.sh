# r05u: the histogram's balanced tile ranges (hb_start) -- GPU tests, then C3 prev/new, C4 prev/new/QE_HIST_TMIN
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/r05u_tests.log 2>&1 || exit 1
REPS=2 timeout -k 10 600 bash tools/gpu_lib_ab.sh r05u_c3 "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
timeout -k 10 900 bash tools/gpu_c4_ab.sh r05u "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "tmin4:QE_HIST_TMIN=4" "tmin8:QE_HIST_TMIN=8" || exit 1
echo all-done
