set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_join_aggregate.py tests/test_gpu_dist.py tests/test_gpu_skew.py -m "gpu and not slow" > gpurun_out/r03f_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_c5.log 2>&1 && \
QE_AGG_BUCKETS=0 timeout -k 10 400 python bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_c5_merge.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_c4.log 2>&1
echo rc=$?
