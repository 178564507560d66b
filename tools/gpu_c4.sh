# sort + golden parity on the GPU, then the C4 batch line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "sort" --timeout 120 --timeout-method thread > gpurun_out/sortpre_tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/golden_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
echo rc=$?
