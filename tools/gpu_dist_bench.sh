# the partitioned plan (C, one RCCL-less rank) and the faithful executor on C3, one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --plan dist --no-cpu > gpurun_out/dist_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/c3_bench.log 2>&1
echo rc=$?
