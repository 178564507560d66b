set -o pipefail
mkdir -p gpurun_out
for v in default ri10 nt384 ri12 default; do
  if [ $v = default ]; then L=""; else L=query-compiler-executor_amd/build/diag/libqe_$v.so; fi
  echo "== $v" >> gpurun_out/kb_sort.log
  QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py sort --reps 8 >> gpurun_out/kb_sort.log 2>&1 || exit 1
done
echo rc=$?
