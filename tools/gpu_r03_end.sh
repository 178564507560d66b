#!/bin/bash
# the round's last GPU call: C3 evidence on the final code (trace + PMC, copied into profiles/ on the
# box, then the bench line), then every -m gpu test, smoke() and every golden
set -o pipefail
mkdir -p gpurun_out
T=${1:-r03zz}
PROFILE_EXTRA=--no-faithful timeout -k 10 600 bash tools/profile_workload.sh ${T} c3 || exit 1
cp gpurun_out/${T}_traffic.json profiles/${T}_traffic.json
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
bash tools/gpu_check_ab.sh || exit 1
echo done
