set -o pipefail
mkdir -p gpurun_out
for v in default b256i2 b512i4 b256i8; do
  if [ $v = default ]; then L=""; else L=query-compiler-executor_amd/build/diag/libqe_$v.so; fi
  echo "== $v" >> gpurun_out/kb_filter.log
  QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py bucket --reps 8 >> gpurun_out/kb_filter.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/kbench.py partition --reps 5 >> gpurun_out/kb_filter.log 2>&1
echo rc=$?
