set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_local_ranks.py tests/test_gpu_comm.py > gpurun_out/r05h_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05h_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "new:QE_NOTHING=1" "res0:QE_P1_RESIDENT=0" "cs3:QE_CS_SINGLE=0" || exit 1
timeout -k 10 900 bash tools/round_end.sh r05h c3 || exit 1
echo all-done
