set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_skew.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_prim_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_single.log 2>&1
echo rc=$?
