# bucket-join load placement variants: same-box A/B on the C3 line (bucket_join stage)
set -o pipefail
mkdir -p gpurun_out
D=query-compiler-executor_amd/build/diag
( for L in "" $D/libqe_HJS.so $D/libqe_HJSX.so $D/libqe_HJSXX.so "" $D/libqe_HJS.so $D/libqe_HJSX.so $D/libqe_HJSXX.so; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], d['roofline']['avg_launch_ms'], json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/hj_bench.log 2>&1
echo rc=$?
