# correctness of the changed kernels (primitives + goldens + comm), then a same-box A/B of one
# environment knob on the C3 bench line:  tools/gpu_r03_ab.sh TAG VAR
set -o pipefail
mkdir -p gpurun_out
T=$1; V=$2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_golden.py -k "not dropin" > gpurun_out/${T}_tests.log 2>&1 && \
bash tools/gpu_env_bench_ab.sh $T $V
echo rc=$?
