#!/bin/bash
# round 3: the batch's shared base-column sorts (qe_sort_cache) and the pipelined histogram --
# parity tests, the C4 bench line (with the no-cache leg beside it), a same-box C3 A/B against
# build/diag/libqe_PREV.so, then the C3 rocprofv3 trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_sort_cache.py \
    tests/test_gpu_golden.py -k "sort_cache or c4_full or (dropin and (c4 or headline or protocol))" \
    > gpurun_out/r03_cache_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c4 --no-cpu > gpurun_out/r03_c4_cache_bench.log 2>&1 || exit 1
bash tools/gpu_lib_ab.sh r03_hist_pipe "new:QE_X=1" "prev:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_PREV.so" || exit 1
PROFILE_EXTRA=--no-faithful timeout -k 10 600 bash tools/profile_workload.sh ${1:-r03c} c3 || exit 1
echo done
