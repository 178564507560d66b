#!/bin/bash
# One same-box A/B gpurun call (replaces round 5's one-off ab_r05*.sh scripts):
#   [TESTS="tests/a.py tests/b.py"] [TEST_LIB=path/libqe_X.so] [REPS=N] \
#       tools/gpu_ab.sh TAG c3|c4|c3c4|none "label:ENV..." ...
# (a variant build is a spec whose ENV sets QE_LIB_PATH=; QE_NOTHING=1 is the product as built)
#   1. TESTS (if set): those -m gpu tests, on the product or on TEST_LIB  -> gpurun_out/TAG_tests.log
#   2. c3: every spec on the C3 line, interleaved REPS (default 2) times   -> gpurun_out/TAG_c3_bench.log
#   3. c4: every spec on the C4 batch line, twice                           -> gpurun_out/TAG_c4.log
# Read-only rocm-smi clock / power / temperature samples every ~2 s run beside it all
# -> gpurun_out/TAG_clocks.log (which box state the numbers were measured in).
# Every GPU step has its own time limit and the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
T=$1; W=$2; shift 2
( while true; do echo "t=$(date +%s)"; rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|junction"; sleep 2; done ) > gpurun_out/${T}_clocks.log 2>&1 &
SMI=$!
trap 'kill $SMI 2>/dev/null' EXIT
if [ -n "$TESTS" ]; then
  env ${TEST_LIB:+QE_LIB_PATH=$TEST_LIB} timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 300 \
      --timeout-method thread $TESTS > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; exit 1; }
fi
case "$W" in *c3*) timeout -k 10 900 bash tools/gpu_lib_ab.sh ${T}_c3 "$@" || exit 1 ;; esac
case "$W" in *c4*) timeout -k 10 900 bash tools/gpu_c4_ab.sh ${T} "$@" || exit 1 ;; esac
echo all-done
