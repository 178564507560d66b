# one C3 bench line (plan executor at N=1) + the GPU tests the plan path touches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bq_bench.json 2> gpurun_out/bq_bench.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_primitives.py > gpurun_out/bq_tests.log 2>&1 || exit 1
echo done
