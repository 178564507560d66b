# end-of-round GPU evidence in one call: every -m gpu test (goldens included), then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/gpu_tests_a.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || exit 1
echo done
