#!/bin/bash
# pass 2's staged 32-bit payloads (XS): the plan / full-size / golden parity tests, then the C3
# line A/B (QE_X32_STAGE) and the C4 line A/B
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_x32s}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_comm.py \
    tests/test_gpu_fullsize.py tests/test_gpu_golden.py -k "comm or c3 or (dropin and (headline or fuzz_a or c4))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh ${T} "staged:QE_X=1" "slotdest:QE_X32_STAGE=0" || exit 1
( for rep in 1 2; do for spec in "staged:QE_X=1" "slotdest:QE_X32_STAGE=0"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])" || exit 1
  done; done ) > gpurun_out/${T}_c4.log 2>&1 || exit 1
echo done
