# XCD-contiguous tiles for the lookback-free passes: same-box A/B against item = blockIdx (NOXCD build)
set -o pipefail
mkdir -p gpurun_out
V=query-compiler-executor_amd/build/diag/libqe_NOXCD.so
run() { echo "== $*"; env "$@" QE_SORT_PIPE=0 QE_PROF_SPLIT=1 timeout -k 10 200 python tools/kbench.py sort --reps 8 2>&1 | grep -v amdgpu.ids | grep -E "pass|hist|local" || return 1; }
( run QE_X=1 && run QE_LIB_PATH=$V && run QE_X=1 && run QE_LIB_PATH=$V && run QE_SORT_PIPE=1 ) > gpurun_out/px_kb.log 2>&1 || exit 1
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_SORT_PIPE=0 QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/px_bench.log 2>&1
echo rc=$?
