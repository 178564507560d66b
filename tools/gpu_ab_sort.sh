# same-box A/B of a variant build on the sort alone (second pass timed on its own) + the C3 line
set -o pipefail
mkdir -p gpurun_out
V=query-compiler-executor_amd/build/diag/libqe_$1.so
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_PROF_SPLIT=1 QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py sort --reps 6 2>&1 | grep -v amdgpu.ids || exit 1; done ) > gpurun_out/ab_kb.log 2>&1 && \
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['config']['stdout'].split()[-1])" || exit 1; done ) > gpurun_out/ab_bench.log 2>&1
echo rc=$?
