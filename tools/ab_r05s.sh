set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/r05s_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05s "hash:QE_NOTHING=1" "merge:QE_HASH_JOIN=0" || exit 1
echo all-done
