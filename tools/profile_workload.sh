#!/bin/bash
# rocprofv3 evidence for one bench workload (run through gpurun from the repo root):
#   tools/profile_workload.sh TAG c4|c5   -> kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE pass
set -e
TAG=$1; W=$2
# raw traces are large: whatever happens, keep only the summaries (gpurun brings back <= 64 MiB)
trap 'rm -rf "$O/${TAG}_trace" "$O/${TAG}_fetch" "$O/${TAG}_write"' EXIT
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--workload $W --steps 2 --warmup 1 --no-cpu $PROFILE_EXTRA"
# C4: a crash under the profiler leaves the fault address, PC and /proc/self/maps here (tools/crashmaps.c).
# Under the profiler C4 runs ONE lane (QE_WORKERS=1): with eight lanes submitting at once the
# profiler's HSA queue interception has faulted past its own 1 MiB buffer (in the trace
# pass and in the counter pass alike); a kernel's bytes do not depend on the lane count, and the
# C4 line itself is measured without the profiler at eight lanes
[ "$W" = c4 ] && export QE_CRASH_MAPS=$O/${TAG}_crashmaps.txt QE_WORKERS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_trace -o run -- python3 $R/bench.py $A > $O/${TAG}_trace.log 2>&1
# C4's counter passes run without the lanes' HIP-event stage table (QE_BENCH_EVENTS=0): under
# --pmc a lane's hipEventRecord has faulted inside librocprofiler-sdk; the counters
# need no events
PMC_ENV=; [ "$W" = c4 ] && PMC_ENV="QE_BENCH_EVENTS=0"
env $PMC_ENV timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch -o run -- python3 $R/bench.py $A > $O/${TAG}_fetch.log 2>&1
env $PMC_ENV timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write -o run -- python3 $R/bench.py $A > $O/${TAG}_write.log 2>&1
echo profile-done
# summaries on the box (a batch workload's raw traces can exceed what gpurun brings back)
cd $R
python3 tools/stage_stats.py $(find $O/${TAG}_trace -name "*kernel_stats.csv" | head -1) --workload $W \
    --out $O/${TAG}_stage_stats.json --command "rocprofv3 --kernel-trace --stats -- python3 bench.py $A" > /dev/null
cp $(find $O/${TAG}_trace -name "*kernel_stats.csv" | head -1) $O/${TAG}_kernel_stats.csv
TW=$W; [ "$W" = c3 ] && case "$PROFILE_EXTRA" in *--no-faithful*) TW=c3_plan;; esac   # (bench.py's C3 tag)
python3 tools/pmc_traffic.py --fetch $O/${TAG}_fetch --write $O/${TAG}_write --out $O/${TAG}_traffic.json --workload $TW \
    --command "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE -- python3 bench.py $A" > /dev/null
rm -rf $O/${TAG}_trace $O/${TAG}_fetch $O/${TAG}_write
echo summaries-done
