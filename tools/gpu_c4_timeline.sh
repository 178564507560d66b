# C4 timeline: one batch on the lanes under a kernel trace (plan, then faithful), summarised on the box
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ex in plan faithful; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c4tl_$ex -o run -- python3 $R/tools/c4_once.py $O/c4tl_$ex.stamp $ex 8 > $O/c4tl_$ex.log 2>&1 || exit 1
  python3 $R/tools/c4_timeline.py $O/c4tl_$ex $O/c4tl_$ex.stamp > $O/c4tl_$ex.txt || exit 1
  rm -rf $O/c4tl_$ex
done
echo done
