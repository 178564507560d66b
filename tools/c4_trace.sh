set -o pipefail
mkdir -p gpurun_out/r04f
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04f/tr -o run -- python3 $R/bench.py --workload c4 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/r04f/c4_trace.log 2>&1
rc=$?
echo "trace rc=$rc"
cp $(find $R/gpurun_out/r04f/tr -name "*kernel_stats.csv" | head -1) $R/gpurun_out/r04f/c4_kernel_stats.csv 2>/dev/null
rm -rf $R/gpurun_out/r04f/tr
exit $rc
