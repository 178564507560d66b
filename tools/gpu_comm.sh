# the RCCL communicator + partitioned executor tests, then the plan's bench line, on one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_comm.py > gpurun_out/comm_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --plan dist --no-cpu > gpurun_out/dist_bench.log 2>&1 && \
QE_SEMI=0 timeout -k 10 300 python bench.py --plan dist --no-cpu > gpurun_out/dist_bench_nosemi.log 2>&1
echo rc=$?
