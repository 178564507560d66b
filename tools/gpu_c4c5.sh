# plan parity (incl. the aggregate fallback), then the C4 and C5 lines, on one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_comm.py > gpurun_out/comm_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/c4_bench.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/c5_bench.log 2>&1
echo rc=$?
