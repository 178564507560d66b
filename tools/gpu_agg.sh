# aggregate join: unit tests, every golden through the binary with QE_AGG_MIN=0, C5 at 1e9, C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_join_aggregate.py > gpurun_out/agg_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_golden.py -k "agg0 or faithful" >> gpurun_out/agg_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize_batch.py -k c5 >> gpurun_out/agg_tests.log 2>&1 || exit 1
echo done
