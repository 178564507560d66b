# end-of-round GPU evidence, part B: the golden fixtures (executor, binary modes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || exit 1
echo done
