#!/bin/bash
# C4 at full size without the shared sorts (the product default): the plan on 8 lanes (bench.py
# --workload c4, parity against c4_full.json) and the faithful executor (test_gpu_fullsize_batch)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03_c4check}
timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 2 --warmup 1 > gpurun_out/${T}_bench.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_fullsize_batch.py -k c4 \
    > gpurun_out/${T}_tests.log 2>&1 || exit 1
echo done
