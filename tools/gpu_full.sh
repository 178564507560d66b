# the full GPU suite, then the C3 bench line (no CPU leg) and the C4 batch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 240 python bench.py --no-cpu > gpurun_out/bench_c3.log 2>&1 && \
timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1
echo rc=$?
