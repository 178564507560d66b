# the drop-in binary in its three modes over every golden, on one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_golden.py -k dropin > gpurun_out/binary_tests.log 2>&1
echo rc=$?
