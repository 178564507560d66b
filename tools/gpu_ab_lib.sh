# same-box A/B of the default libqe against a variant build: kbench WHAT + the C3 bench line
#   bash tools/gpu_ab_lib.sh VARIANT WHAT
set -o pipefail
mkdir -p gpurun_out
V=query-compiler-executor_amd/build/diag/libqe_$1.so
W=${2:-merge}
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py $W --reps 6 2>&1 | grep -v amdgpu.ids || exit 1; done ) > gpurun_out/ab_kb.log 2>&1 && \
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['stages']['mj_fused'])" || exit 1; done ) > gpurun_out/ab_bench.log 2>&1
echo rc=$?
