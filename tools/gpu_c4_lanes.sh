set -o pipefail
mkdir -p gpurun_out
( for w in 8 12 16 8 12 16; do echo "== QE_WORKERS=$w"; QE_WORKERS=$w timeout -k 10 300 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])" || exit 1; done ) > gpurun_out/r03_c4_lanes.log 2>&1
echo rc=$?
