# C5: aggregate-join tests, then the C5 line with this build vs build/diag/libqe_PREV.so (two rounds)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_join_aggregate.py tests/test_gpu_skew.py tests/test_gpu_fullsize_batch.py > gpurun_out/$1_tests.log 2>&1 || exit 1
for rep in 1 2; do for spec in "new:QE_X=1" "prev:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_PREV.so"; do
  label=${spec%%:*}; envs=${spec#*:}
  echo "== $label" >> gpurun_out/$1_bench.log
  env $envs timeout -k 10 300 python bench.py --workload c5 --no-cpu --steps 3 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stdout'] if 'stdout' in d else '', {k: v['ms_per_step'] for k, v in d.get('stages', {}).items()})" >> gpurun_out/$1_bench.log || exit 1
done; done
echo rc=$?
