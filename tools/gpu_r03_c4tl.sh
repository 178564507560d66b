#!/bin/bash
# C4 with the shared base-column sorts: parity (goldens through the binary, the shared-sort tests,
# the full-size batch), the bench line, then one batch's kernel timeline on the plan lanes
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_c4}
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_sort_cache.py \
    tests/test_gpu_bucket_join.py tests/test_gpu_golden.py -k "sort_cache or bucket_join or (dropin and (c4 or headline or fuzz_a))" \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c4 --no-cpu --warmup 2 > gpurun_out/${T}_bench.log 2>&1 || exit 1
R=$(pwd); O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_tl -o run -- python3 $R/tools/c4_once.py $O/${T}_tl.stamp plan 8 > $O/${T}_tl.log 2>&1 || exit 1
python3 $R/tools/c4_timeline.py $O/${T}_tl $O/${T}_tl.stamp > $O/${T}_timeline.txt || exit 1
rm -rf $O/${T}_tl
echo done
