#!/bin/bash
# the wave-per-bucket local sort: sort / merge / bucket-join / golden parity, then the C4 line A/B
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_histpart}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_primitives.py \
    tests/test_gpu_bucket_join.py tests/test_gpu_sort_cache.py tests/test_gpu_golden.py \
    -k "sort or merge or bucket_join or sort_cache or (dropin and (c4 or fuzz_a or headline))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
( for rep in 1 2; do for spec in "part:QE_X=1" "atomic:QE_HIST_PART=0"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'], {k: (v['ms_per_step'], v['launches_per_step']) for k, v in list(d['stages_lane0'].items())[:6]})" || exit 1
  done; done ) > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo done
