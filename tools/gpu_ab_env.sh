# full GPU suite, then a same-box A/B of one environment knob on the C3 bench line (and C4)
#   bash tools/gpu_ab_env.sh "QE_X=1"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
( for v in "" "$1" "" "$1"; do echo "== ${v:-default}"; env $v timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'])" || exit 1; done ) > gpurun_out/ab_bench.log 2>&1 && \
( for v in "" "$1"; do echo "== ${v:-default}"; env $v timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 2 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])" || exit 1; done ) >> gpurun_out/ab_bench.log 2>&1
echo rc=$?
