set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_local_ranks.py tests/test_gpu_comm.py > gpurun_out/r05f_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05f_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "tm2e:QE_LIB_PATH=$AB/libqe_tm2.so" "tm1:QE_LIB_PATH=$AB/libqe_p1tm1.so" "new:QE_NOTHING=1" "cs3:QE_CS_SINGLE=0" || exit 1
timeout -k 10 900 bash tools/round_end.sh r05f c3 || exit 1
echo all-done
