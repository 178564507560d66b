# pipelined sort passes: parity tests, then same-box A/B (QE_SORT_PIPE=0/1) on the sort and on C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py > gpurun_out/pa_tests.log 2>&1 || exit 1
( for P in 0 1 0 1; do echo "== QE_SORT_PIPE=$P"; QE_SORT_PIPE=$P QE_PROF_SPLIT=1 timeout -k 10 200 python tools/kbench.py sort --reps 6 2>&1 | grep -v amdgpu.ids || exit 1; done ) > gpurun_out/pa_kb.log 2>&1 || exit 1
( for P in 0 1 0 1; do echo "== QE_SORT_PIPE=$P"; QE_SORT_PIPE=$P timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/pa_bench.log 2>&1
echo rc=$?
