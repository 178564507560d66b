# round 6 working call: large-block backing A/B (contiguous pages / one arena) on the C3 line
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06h}
REPS=2 bash tools/gpu_ab.sh $T c3 "base:QE_NOTHING=1" "contig:QE_ALLOC_CONTIG=1" "arena:QE_ALLOC_ARENA_GB=48" || exit 1
echo all-done
