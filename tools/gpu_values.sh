# select values carried instead of rowids (+ the aggregate last join): the plan's GPU tests, then a
# same-box A/B of bench.py against QE_PLAN_VALUES=0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_bucket_join.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/values_tests.log 2>&1 || exit 1
( for A in 1 0 1 0; do echo "== QE_PLAN_VALUES=$A"; QE_PLAN_VALUES=$A timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['host_round_trips_per_step'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1; done ) > gpurun_out/values_ab.log 2>&1
echo rc=$?
