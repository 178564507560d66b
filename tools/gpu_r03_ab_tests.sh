set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_local_ranks.py tests/test_gpu_bucket_join.py > gpurun_out/ko_local.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_golden.py tests/test_gpu_dist.py > gpurun_out/ko_golden.log 2>&1 && \
bash tools/gpu_lib_ab.sh ko "new:QE_X=1" "prev:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_PREV.so"
echo rc=$?
