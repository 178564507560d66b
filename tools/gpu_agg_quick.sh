# aggregate join unit tests + C5 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_join_aggregate.py > gpurun_out/agg_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err || exit 1
echo done
