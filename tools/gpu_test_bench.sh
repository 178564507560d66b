# the sort / join GPU tests, then the default C3 bench line (no CPU leg)
set -o pipefail
mkdir -p gpurun_out
T=${1:-tb}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_fullsize.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo done
