# the next-join-key carry: the plan's device paths (in-process ranks W = 2, 3, 8 on every golden and
# at 100 M, the goldens in every mode, the dist / full-size parity) then an on/off A/B of the C3 line
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_local_ranks.py > gpurun_out/kc_local.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_golden.py tests/test_gpu_dist.py > gpurun_out/kc_golden.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_fullsize.py tests/test_gpu_bucket_join.py > gpurun_out/kc_full.log 2>&1 && \
bash tools/gpu_lib_ab.sh kc "on:QE_X=1" "off:QE_PLAN_KEY_CARRY=0"
echo rc=$?
