set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_local_ranks.py tests/test_gpu_fullsize.py tests/test_gpu_skew.py tests/test_gpu_sort_cache.py > gpurun_out/r05m_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05m_c3 "new:QE_NOTHING=1" "k64:QE_GATHER_K32=0" || exit 1
timeout -k 10 600 bash tools/gpu_c4_ab.sh r05m "new:QE_NOTHING=1" "k64:QE_GATHER_K32=0" || exit 1
echo all-done
