# the plan's last join in aggregate form: the comm/plan GPU tests (every golden through
# qe_run_queries_dist, the 75 M / 100 M cases), then a same-box A/B against QE_PLAN_AGG=0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_comm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/agg_last_tests.log 2>&1 || exit 1
( for A in 1 0 1 0; do echo "== QE_PLAN_AGG=$A"; QE_PLAN_AGG=$A timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['host_round_trips_per_step'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1; done ) > gpurun_out/agg_last_ab.log 2>&1
echo rc=$?
