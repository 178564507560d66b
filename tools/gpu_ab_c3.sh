# same-box A/B of a variant build on the C3 bench line, with the stages that differ
set -o pipefail
mkdir -p gpurun_out
V=query-compiler-executor_amd/build/diag/libqe_$1.so
( for L in "" $V "" $V; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'], d['config']['stdout'].split()[-1]); [print('   ', k, v['ms_per_step']) for k, v in d['stages'].items() if k in sys.argv[1:]]" ${@:2} || exit 1; done ) > gpurun_out/ab_bench.log 2>&1
echo rc=$?
