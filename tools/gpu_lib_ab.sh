# same-box A/B of library builds (and env settings) on the C3 bench line:
#   tools/gpu_lib_ab.sh TAG "LABEL:ENV..." ...   (ENV: VAR=V pairs, QE_LIB_PATH= for a variant build)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
( for rep in $(seq ${REPS:-2}); do for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1
  done; done ) > gpurun_out/${T}_bench.log 2>&1
echo rc=$?
