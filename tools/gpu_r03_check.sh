# round 3 check: the in-process ranks (W = 2, 3, 8) on every golden and at 100 M, the drop-in
# binary in every mode, the comm / parallel tests
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_local_ranks.py -m "gpu and not slow" > gpurun_out/r03_local.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_golden.py > gpurun_out/r03_golden.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_comm.py tests/test_gpu_parallel.py -m "gpu and not slow" > gpurun_out/r03_comm.log 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_local_ranks.py -m "gpu and slow" > gpurun_out/r03_local_slow.log 2>&1
echo rc=$?
