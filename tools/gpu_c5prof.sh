# C5 kernel trace (aggregate join): per-kernel durations
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o c5 -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/c5prof.log 2>&1 || exit 1
find gpurun_out/c5prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c5_kernel_stats.csv
echo done
