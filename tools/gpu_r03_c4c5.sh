set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_c4.log 2>&1 && \
timeout -k 10 400 python bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_c5.log 2>&1
echo rc=$?
