# round evidence on one MI355X: the default bench line, then rocprofv3 kernel trace + stats and
# the two PMC passes of the same C3 command (tools/profile_round.sh)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-prof}
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 && \
bash tools/profile_round.sh ${TAG}
echo rc=$?
