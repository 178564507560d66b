# GPU tests of the sort / join paths, then same-box A/B of the working tree against a build of HEAD
# (build/diag/libqe_HEAD.so): the sort passes (kbench) and the C3 line
set -o pipefail
mkdir -p gpurun_out
T=${1:-ah}
V=query-compiler-executor_amd/build/diag/libqe_HEAD.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_fullsize.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
( for L in "" $V "" $V; do echo "== ${L:-work}"; QE_PROF_SPLIT=1 QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py sort --reps 8 2>&1 | grep -E "pass|hist" || exit 1; done ) > gpurun_out/${T}_kb.log 2>&1 || exit 1
( for L in "" $V "" $V; do echo "== ${L:-work}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['roofline']['avg_launch_ms'], json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/${T}_bench.log 2>&1
echo rc=$?
