# round 6 working call: side-stream parity at 100 M, the cost-model inputs, C3 A/B with clocks
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06e}
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "side_stream or c3" > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/cost_constants.py > gpurun_out/${T}_cost_constants.json 2> gpurun_out/${T}_cost_constants.err || exit 1
REPS=2 bash tools/gpu_ab.sh $T c3 "base:QE_NOTHING=1" "sums1:QE_HJ_SUMS_FORM=1" "sums2:QE_HJ_SUMS_FORM=2" "fork:QE_SIDE_STREAM=1" || exit 1
echo all-done
