#!/bin/bash
# one GPU call: the named GPU tests, then a same-box A/B of build/var/libqe_PREV.so (the last
# commit's build) against the product on the C3 line, then the C3 rocprofv3 trace + PMC passes
#   tools/check_then_ab.sh TAG tests/test_a.py tests/test_b.py ...
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_tests.log 2>&1 || exit 1
fi
bash tools/gpu_lib_ab.sh ${T}_ab "prev:QE_LIB_PATH=$PWD/query-compiler-executor_amd/build/var/libqe_PREV.so" "new:QE_NOTHING=1" || exit 1
PROFILE_EXTRA=--no-faithful timeout -k 10 600 bash tools/profile_workload.sh ${T} c3 || exit 1
echo all-done
