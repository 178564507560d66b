# the concurrent batch executor: its tests, then the C4 line, on one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parallel.py > gpurun_out/par_tests.log 2>&1 && \
for w in 2 4 8; do QE_WORKERS=$w timeout -k 10 300 python bench.py --workload c4 --no-cpu > gpurun_out/c4_w$w.log 2>&1 || exit 1; done
echo rc=$?
