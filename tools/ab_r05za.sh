# r05za: the aggregate-form bucket join as a resident grid (default) vs one workgroup per bucket (QE_HJ_SUMS_PERSIST=0), C3
set -o pipefail
mkdir -p gpurun_out
REPS=3 timeout -k 10 700 bash tools/gpu_lib_ab.sh r05za_c3 "persist:QE_NOTHING=1" "perbucket:QE_HJ_SUMS_PERSIST=0" || exit 1
echo all-done
