# the RCCL communicator + partitioned executor tests on one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_comm.py > gpurun_out/comm_tests.log 2>&1
echo rc=$?
