# C4 and C5 bench lines with the current library (no CPU leg)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c4 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03d_c4_bench.json 2> gpurun_out/r03d_c4.err && \
timeout -k 10 400 python bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/r03d_c5_bench.json 2> gpurun_out/r03d_c5.err
echo rc=$?
