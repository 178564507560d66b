#!/bin/bash
# the chain bucket join as a resident grid: parity (bucket join, plan, goldens, full-size C3), then
# the C3 line and the C4 line A/B'd on QE_HJ_PERSIST, same box
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_hjpersist}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_bucket_join.py \
    tests/test_gpu_comm.py tests/test_gpu_fullsize.py tests/test_gpu_sort_cache.py tests/test_gpu_golden.py \
    -k "bucket_join or comm or c3 or sort_cache or (dropin and (headline or fuzz_a or c4))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh ${T}_c3 "persist:QE_HJ_PERSIST=1" "perbucket:QE_HJ_PERSIST=0" || exit 1
( for rep in 1 2; do for spec in "persist:QE_HJ_PERSIST=1" "perbucket:QE_HJ_PERSIST=0"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'], {k: (v['ms_per_step'], v['launches_per_step']) for k, v in list(d['stages_lane0'].items())[:6]})" || exit 1
  done; done ) > gpurun_out/${T}_c4_bench.log 2>&1 || exit 1
echo done
