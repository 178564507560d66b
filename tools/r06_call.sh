# round 6 working call: the fused scan emitting the join-key values (QE_SCAN_KEYS): GPU tests, C3 A/B
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06m}
TESTS="tests/test_gpu_comm.py tests/test_gpu_local_ranks.py tests/test_gpu_fullsize.py" \
REPS=2 bash tools/gpu_ab.sh $T c3 "keys:QE_NOTHING=1" "gather:QE_SCAN_KEYS=0" || exit 1
echo all-done
