#!/bin/bash
# per-phase stamps of every lookback-free first pass and every second pass of one C3 query
# (a -DQE_DIAG_STAMPS build: tools/build_variant.sh STAMPS "-DQE_DIAG_STAMPS"), one run per launch
#   tools/stamps_c3.sh TAG   -> gpurun_out/TAG_stamps.log
set -o pipefail
mkdir -p gpurun_out
T=${1:-stamps}
export QE_LIB_PATH=${QE_LIB_PATH:-$PWD/query-compiler-executor_amd/build/var/libqe_STAMPS.so}
( for k in 1 2 3 4 5 6; do
    echo "=== p1:$k"; QE_STAMP_SEL=p1:$k timeout -k 10 120 python tools/stamps.py --what c3p1 2>&1 | grep -v "^\[stamps\] p2" || exit 1
  done
  for k in 1 2 3 4 5 6; do
    echo "=== p2:$k"; QE_STAMP_SEL=p2:$k timeout -k 10 120 python tools/stamps.py --what c3p2 2>&1 | grep -v "^\[stamps\] p1" || exit 1
  done ) > gpurun_out/${T}_stamps.log 2>&1
rc=$?
echo stamps rc=$rc
exit $rc
