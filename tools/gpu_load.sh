# loader (f-3): parity through the goldens (every golden loads its relations from host memory),
# then the host -> HBM rate at 8 and 1 staging threads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/golden_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/loadbench.py --reps 2 > gpurun_out/loadbench.log 2>&1 && \
QE_LOAD_THREADS=1 timeout -k 10 400 python -u tools/loadbench.py --reps 1 > gpurun_out/loadbench_t1.log 2>&1
echo rc=$?
