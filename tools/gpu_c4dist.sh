set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_golden.py -k "c4_replicas or lanes4 or agg_plan" > gpurun_out/c4dist_tests.log 2>&1
echo rc=$?
