# round 3: C5-in-plan tests + the changed kernels' tests, then A/Bs: pipelined wave scan, chain bucket join
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_dist.py tests/test_gpu_local_ranks.py tests/test_gpu_skew.py tests/test_gpu_join_aggregate.py -m "gpu and not slow" > gpurun_out/r03c_tests.log 2>&1 && \
bash tools/gpu_env_bench_ab.sh r03wsp2 QE_WSPIPE && \
bash tools/gpu_env_bench_ab.sh r03chain QE_HJ_CHAIN && \
QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_STAMPS.so timeout -k 10 120 python tools/stamps.py --what cp > gpurun_out/r03_wsp_stamps.log 2>&1
echo rc=$?
