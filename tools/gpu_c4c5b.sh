# the C4 and C5 bench lines with the round's final code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/c4_final.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/c5_final.log 2>&1 || exit 1
echo done
