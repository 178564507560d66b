# r05v: the single-block bucket scans with coalesced global accesses (rows_in / rows_out) -- GPU tests, C3 and C4 new/prev
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/r05v_tests.log 2>&1 || exit 1
REPS=2 timeout -k 10 600 bash tools/gpu_lib_ab.sh r05v_c3 "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05v "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
echo all-done
