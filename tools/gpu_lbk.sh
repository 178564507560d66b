# wide lookback: primitives tests, then the filter kbench over lookback widths (LB_K 4 default, 1, 8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_primitives.py > gpurun_out/lbk_tests.log 2>&1 || exit 1
for v in default lbk1 lbk8 default; do
  if [ $v = default ]; then L=""; else L=query-compiler-executor_amd/build/diag/libqe_$v.so; fi
  echo "== $v" >> gpurun_out/lbk_kb.log
  QE_LIB_PATH=$L timeout -k 10 200 python tools/kbench.py filter --reps 8 >> gpurun_out/lbk_kb.log 2>&1 || exit 1
done
echo done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_bucket_join.py >> gpurun_out/lbk_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/lbk_bench.json 2> gpurun_out/lbk_bench.err || exit 1
echo done2
