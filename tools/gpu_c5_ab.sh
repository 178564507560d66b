# aggregate-join GPU tests, then a same-box A/B of the C5 line against build/diag/libqe_HEAD.so
set -o pipefail
mkdir -p gpurun_out
T=${1:-c5ab}
V=query-compiler-executor_amd/build/diag/libqe_HEAD.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_join_aggregate.py tests/test_gpu_skew.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
( for L in "" $V "" $V; do echo "== ${L:-work}"; QE_LIB_PATH=$L timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['stdout'].strip(), json.dumps(d['stages']))" || exit 1; done ) > gpurun_out/${T}_bench.log 2>&1
echo rc=$?
