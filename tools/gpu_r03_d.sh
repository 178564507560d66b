# round 3: the unordered plan scan -- goldens through the plan (binary + dist + local ranks), A/B
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_comm.py tests/test_gpu_local_ranks.py tests/test_gpu_golden.py -k "dist or local or dropin" > gpurun_out/r03d_tests.log 2>&1 && \
bash tools/gpu_env_bench_ab.sh r03uscan QE_PLAN_USCAN
echo rc=$?
