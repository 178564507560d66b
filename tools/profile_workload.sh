#!/bin/bash
# rocprofv3 evidence for one bench workload (run through gpurun from the repo root):
#   tools/profile_workload.sh TAG c4|c5   -> kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE pass
set -e
TAG=$1; W=$2
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--workload $W --steps 2 --warmup 1 --no-cpu"
export QE_BENCH_EVENTS=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_trace -o run -- python3 $R/bench.py $A > $O/${TAG}_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch -o run -- python3 $R/bench.py $A > $O/${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write -o run -- python3 $R/bench.py $A > $O/${TAG}_write.log 2>&1
echo profile-done
