# round 6 working call: the fused scan's key loads issued with the predicate columns (every row) vs
# by the surviving lanes after the predicate
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06n}
V=$PWD/query-compiler-executor_amd/build/var
REPS=2 bash tools/gpu_ab.sh $T c3 "late:QE_NOTHING=1" "early:QE_LIB_PATH=$V/libqe_kearly.so" || exit 1
echo all-done
