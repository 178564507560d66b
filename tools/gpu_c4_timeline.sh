# C4 timeline: one batch on the lanes under a kernel trace (default: plan, then faithful), summarised
# on the box; a crash leaves its fault address, PC and /proc/self/maps in c4tl_EX.crashmaps.txt
#   tools/gpu_c4_timeline.sh [TAG] [executors...]
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
T=${1:-c4tl}; shift
EXS=${*:-plan faithful}
cd /tmp && export TMPDIR=/tmp
for ex in $EXS; do
  QE_CRASH_MAPS=$O/${T}_$ex.crashmaps.txt timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_$ex -o run -- python3 $R/tools/c4_once.py $O/${T}_$ex.stamp $ex 8 > $O/${T}_$ex.log 2>&1 || exit 1
  python3 $R/tools/c4_timeline.py $O/${T}_$ex $O/${T}_$ex.stamp > $O/${T}_$ex.txt || exit 1
  rm -rf $O/${T}_$ex
done
echo done
