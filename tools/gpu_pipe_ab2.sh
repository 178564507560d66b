# pipelined sort passes: mapping / grid variants on the sort (same box)
set -o pipefail
mkdir -p gpurun_out
S=query-compiler-executor_amd/build/diag/libqe_STRIDE.so
run() { echo "== $*"; env "$@" QE_PROF_SPLIT=1 timeout -k 10 200 python tools/kbench.py sort --reps 6 2>&1 | grep -v amdgpu.ids | grep -E "pass|pipe grid" || return 1; }
( run QE_SORT_PIPE=0 && run QE_SORT_PIPE=1 QE_PIPE_DEBUG=1 && run QE_SORT_PIPE=1 QE_PIPE_BPC=2 && run QE_SORT_PIPE=1 QE_LIB_PATH=$S && run QE_SORT_PIPE=1 QE_LIB_PATH=$S QE_PIPE_BPC=3 && run QE_SORT_PIPE=0 ) > gpurun_out/pb_kb.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 > gpurun_out/pb_bench.json 2> gpurun_out/pb_bench.err
echo rc=$?
