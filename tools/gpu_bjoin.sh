# the bucket join: its tests, the plan's golden parity, then the plan bench vs the merge form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucket_join.py tests/test_gpu_comm.py > gpurun_out/bjoin_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/dist_bench.log 2>&1
echo rc=$?
