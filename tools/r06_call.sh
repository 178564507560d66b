# round 6 working call: the box's clock state under the C3 loop, then the GPU tests of the new paths
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06f}
timeout -k 10 400 bash tools/clock_probe.sh $T 400 || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_local_ranks.py tests/test_gpu_bucket_join.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no-cpu --steps 10 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo all-done
