# same-box A/B of one environment knob on the C3 bench line (no tests):
#   tools/gpu_env_bench_ab.sh TAG VAR   (VAR=1 vs VAR=0, twice each)
set -o pipefail
mkdir -p gpurun_out
T=$1; V=$2
( for E in "$V=1" "$V=0" "$V=1" "$V=0"; do echo "== $E"; env $E timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1; done ) > gpurun_out/${T}_bench.log 2>&1
echo rc=$?
