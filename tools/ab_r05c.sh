set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_bucket_join.py tests/test_gpu_comm.py tests/test_gpu_local_ranks.py > gpurun_out/r05c_tests.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh r05c_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "noprerank_noflat:QE_LIB_PATH=$AB/libqe_noprerank.so" "p1only:QE_LIB_PATH=$AB/libqe_p1only.so" "p2only:QE_LIB_PATH=$AB/libqe_p2only.so" "p1late:QE_LIB_PATH=$AB/libqe_p1late.so" "new_flat:QE_NOTHING=1" "new_flat_hj1:QE_HJ8=0" || exit 1
bash tools/gpu_c4_ab.sh r05c "new_flat:QE_NOTHING=1" "new_flat_hj1:QE_HJ8=0" || exit 1
echo all-done
