#!/bin/bash
# End-of-round evidence, split so each part fits one gpurun call (run from the repo root):
#   tools/round_end.sh TAG c3     -> C3 rocprofv3 trace + PMC passes, then `python bench.py` (the line
#                                    picks the fresh per-query traffic: copied to profiles/ first)
#   tools/round_end.sh TAG c45    -> the same for C5, then for C4
#   tools/round_end.sh TAG c4     -> the C4 line, then its trace + PMC passes (best effort)
#   tools/round_end.sh TAG check  -> every -m gpu test, smoke(), the goldens (tools/gpu_check_ab.sh)
set -o pipefail
mkdir -p gpurun_out
T=$1
case "$2" in
c3)
  PROFILE_EXTRA=--no-faithful timeout -k 10 700 bash tools/profile_workload.sh ${T} c3 || exit 1
  cp gpurun_out/${T}_traffic.json profiles/${T}_traffic.json || exit 1
  timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
  ;;
c45)
  timeout -k 10 500 bash tools/profile_workload.sh ${T}c5 c5 || exit 1
  cp gpurun_out/${T}c5_traffic.json profiles/${T}c5_traffic.json || exit 1
  timeout -k 10 300 python bench.py --workload c5 > gpurun_out/${T}_c5_bench.json 2> gpurun_out/${T}_c5_bench.err || exit 1
  # C4: the bench line first, then its profile (best effort: see the c4 case)
  timeout -k 10 400 python bench.py --workload c4 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || exit 1
  timeout -k 10 500 bash tools/profile_workload.sh ${T}c4 c4 || echo "c4 profile failed (rc $?)"
  ;;
c4)
  # the bench line first (no profiler), then the trace + PMC passes as best effort: the 8 lanes'
  # HIP calls under rocprofv3's kernel trace have crashed inside the runtime
  timeout -k 10 400 python bench.py --workload c4 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || exit 1
  timeout -k 10 600 bash tools/profile_workload.sh ${T}c4 c4 || echo "c4 profile failed (rc $?)"
  ;;
check)
  bash tools/gpu_check_ab.sh || exit 1
  ;;
*) echo "usage: $0 TAG c3|c45|c4|check"; exit 2 ;;
esac
echo round-end-$2-done
