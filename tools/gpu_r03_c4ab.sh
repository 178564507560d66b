#!/bin/bash
# C4 parity (goldens through the binary, the shared-sort tests, the full-size batch) then the C4
# bench line A/B'd against env knobs on the same box:  tools/gpu_r03_c4ab.sh TAG "label:ENV=V ..." ...
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_sort_cache.py \
    tests/test_gpu_golden.py -k "sort_cache or (dropin and (c4 or headline or fuzz_a))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
( for rep in 1 2; do for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'], d.get('sort_cache'), {k: (v['ms_per_step'], v['launches_per_step']) for k, v in d['stages_lane0'].items()})" || exit 1
  done; done ) > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo done
