# the plan's GPU parity tests (in-process ranks incl. 100 M, bucket join, goldens, dist, full size)
# then an A/B of the C3 line against build/diag/libqe_PREV.so.  TAG: $1
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_local_ranks.py tests/test_gpu_bucket_join.py > gpurun_out/$1_local.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_golden.py tests/test_gpu_dist.py > gpurun_out/$1_golden.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_fullsize.py > gpurun_out/$1_full.log 2>&1 && \
bash tools/gpu_lib_ab.sh $1 "new:QE_X=1" "prev:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_PREV.so"
echo rc=$?
