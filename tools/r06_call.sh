# round 6 working call: the chain join in 512-thread workgroups (three per CU) vs 1024 (two)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06q}
QE_HJ_NT512=1 timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_bucket_join.py tests/test_gpu_fullsize.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
REPS=2 bash tools/gpu_ab.sh $T c3 "base:QE_NOTHING=1" "nt512:QE_HJ_NT512=1" || exit 1
echo all-done
