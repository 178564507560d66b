# round evidence: C3 bench line + rocprofv3 trace + PMC passes (tools/gpu_profile.sh TAG), then the
# C4 and C5 lines
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01e}
bash tools/gpu_profile.sh $TAG > gpurun_out/${TAG}_profile.out 2>&1 && \
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/${TAG}_c4.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/${TAG}_c5.log 2>&1
echo rc=$?
