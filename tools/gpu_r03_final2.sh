#!/bin/bash
# round-3 evidence, C4 and C5: the C5 trace + PMC passes (copied into profiles/ on the box so the
# C5 line carries them), the C5 line, then the C4 line (C4 under rocprofv3's kernel trace crashed
# inside the HIP runtime's event polling; its timeline comes from tools/gpu_r03_c4tl.sh)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03z}
timeout -k 10 600 bash tools/profile_workload.sh ${T}c5 c5 || exit 1
cp gpurun_out/${T}c5_traffic.json profiles/${T}c5_traffic.json
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/${T}_c5_bench.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c4 --warmup 2 > gpurun_out/${T}_c4_bench.log 2>&1 || exit 1
echo done
