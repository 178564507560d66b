set -o pipefail
mkdir -p gpurun_out
( for q in 4 8 16; do for w in 8 16; do echo "== GPU_MAX_HW_QUEUES=$q QE_WORKERS=$w"; GPU_MAX_HW_QUEUES=$q QE_WORKERS=$w timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])" || exit 1; done; done ) > gpurun_out/r03_c4_queues.log 2>&1
echo rc=$?
