# same-box A/B of filter-scan tile shapes (tools/build_variant.sh builds them)
set -o pipefail
mkdir -p gpurun_out
for v in default fs16 fs12 default fs16 fs12; do
  if [ $v = default ]; then L=""; else L=query-compiler-executor_amd/build/var/libqe_$v.so; fi
  echo "== $v" >> gpurun_out/kb_filter.log
  QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py filter --reps 8 >> gpurun_out/kb_filter.log 2>&1 || exit 1
done
echo rc=$?
