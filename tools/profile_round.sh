#!/bin/bash
# rocprofv3 evidence for bench.py on one MI355X (run through gpurun from the repo root):
#   1. kernel trace + stats   2. FETCH_SIZE pass   3. WRITE_SIZE pass (counters in their own runs,
#   no sys/runtime trace beside --pmc).  Outputs under gpurun_out/$TAG*.
set -e
TAG=${1:-prof}
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-faithful > $O/${TAG}_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-faithful > $O/${TAG}_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-faithful > $O/${TAG}_write.log 2>&1
echo profile-done
