#!/bin/bash
# the aggregate last join's persistent form: its parity tests, then the C3 line A/B (QE_HJ_SUMS_PERSIST)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_sums}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_comm.py \
    tests/test_gpu_fullsize.py tests/test_gpu_golden.py -k "comm or c3 or (dropin and (headline or fuzz_a or c4))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh ${T} "persist:QE_HJ_SUMS_PERSIST=1" "perbucket:QE_HJ_SUMS_PERSIST=0" || exit 1
echo done
