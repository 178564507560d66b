#!/bin/bash
# C4 knobs: the shared-sort tests (goldens + full batch) with QE_JOIN_UNIFY=1, then the C4 bench
# line A/B'd over "label:ENV=V ..." specs on the same box (two rounds)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_primitives.py \
    -k "unsorted" > gpurun_out/${T}_tests.log 2>&1 || exit 1
QE_JOIN_UNIFY=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_sort_cache.py >> gpurun_out/${T}_tests.log 2>&1 || exit 1
( for rep in 1 2; do for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'], {k: (v['ms_per_step'], v['launches_per_step']) for k, v in list(d['stages_lane0'].items())[:6]})" || exit 1
  done; done ) > gpurun_out/${T}_bench.log 2>&1 || exit 1
echo done
