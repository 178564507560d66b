# r05w: the chain bucket join walking buckets with the next bucket's bounds in flight (QE_HJ_PERSIST) -- GPU tests, C3 and C4 on/off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_golden.py > gpurun_out/r05w_tests.log 2>&1 || exit 1
REPS=2 timeout -k 10 600 bash tools/gpu_lib_ab.sh r05w_c3 "persist:QE_NOTHING=1" "grid32k:QE_HJ_PERSIST=0" || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05w "persist:QE_NOTHING=1" "grid32k:QE_HJ_PERSIST=0" || exit 1
echo all-done
