# C3 plan: bench line, then a kernel trace of a few steps (inter-kernel idle time per query)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/gaps_bench.json 2> gpurun_out/gaps_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps_trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-faithful > gpurun_out/gaps_trace.log 2>&1 || exit 1
echo done
