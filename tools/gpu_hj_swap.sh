# bucket join with the smaller side in LDS: bucket-join + plan GPU tests, then a same-box A/B of
# bench.py against QE_HJ_SWAP=0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_bucket_join.py tests/test_gpu_comm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hj_swap_tests.log 2>&1 || exit 1
( for A in 1 0 1 0; do echo "== QE_HJ_SWAP=$A"; QE_HJ_SWAP=$A timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1; done ) > gpurun_out/hj_swap_ab.log 2>&1
echo rc=$?
