# fused per-bucket join: its tests, the whole GPU suite, then a same-box A/B (QE_FUSED_JOIN=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_join.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fused_tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
( for v in "" "QE_FUSED_JOIN=1"; do echo "== ${v:-default}"; env $v timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['config']['stdout'].split()[-1]); [print('   ', k, v['ms_per_step'], v['launches_per_step']) for k, v in list(d['stages'].items())[:8]]" || exit 1; done ) > gpurun_out/ab_bench.log 2>&1
echo rc=$?
