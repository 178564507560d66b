# payload carry through the sort + bucket join: plan GPU tests, then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_bucket_join.py > gpurun_out/carry_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/carry_bench.json 2> gpurun_out/carry_bench.err || exit 1
echo done
