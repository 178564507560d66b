#!/bin/bash
# round-3 evidence on one box: per workload the rocprofv3 kernel trace + the two PMC passes
# (tools/profile_workload.sh), copied into profiles/ on the box so the bench line that follows
# carries this box's traffic, then the bench line itself (C3 default with the CPU baseline, C4, C5)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03z}
PROFILE_EXTRA=--no-faithful timeout -k 10 600 bash tools/profile_workload.sh ${T} c3 || exit 1
cp gpurun_out/${T}_traffic.json profiles/${T}_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
PROFILE_EXTRA="--warmup 2" timeout -k 10 600 bash tools/profile_workload.sh ${T}c4 c4 || exit 1
cp gpurun_out/${T}c4_traffic.json profiles/${T}c4_traffic.json
timeout -k 10 400 python bench.py --workload c4 --warmup 2 > gpurun_out/${T}_c4_bench.log 2>&1 || exit 1
timeout -k 10 600 bash tools/profile_workload.sh ${T}c5 c5 || exit 1
cp gpurun_out/${T}c5_traffic.json profiles/${T}c5_traffic.json
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/${T}_c5_bench.log 2>&1 || exit 1
echo done
