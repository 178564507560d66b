# round 6 working call: GPU tests of the touched paths, C3 A/B of the side stream, the C4 line
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06d}
TESTS="tests/test_gpu_comm.py tests/test_gpu_local_ranks.py tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_fullsize.py" \
  REPS=2 bash tools/gpu_ab.sh $T c3 "fork:QE_NOTHING=1" "nofork:QE_SIDE_STREAM=0" || exit 1
timeout -k 10 400 python bench.py --workload c4 --no-cpu > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || exit 1
echo all-done
