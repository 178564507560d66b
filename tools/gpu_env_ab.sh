# plan-path GPU tests, then a same-box A/B of one environment knob on the C3 line:
#   tools/gpu_env_ab.sh TAG VAR   (VAR=0 vs VAR unset, twice each)
set -o pipefail
mkdir -p gpurun_out
T=$1; V=$2
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucket_join.py tests/test_gpu_comm.py tests/test_gpu_fullsize.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
( for E in "$V=1" "$V=0" "$V=1" "$V=0"; do echo "== $E"; env $E timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/${T}_bench.log 2>&1
echo rc=$?
