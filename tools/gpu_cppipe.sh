# pipelined compaction: primitives tests, then filter kbench pipelined vs one tile per workgroup
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_primitives.py > gpurun_out/cppipe_tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  echo "== QE_CP_PIPE=$v" >> gpurun_out/cppipe_kb.log
  QE_CP_PIPE=$v timeout -k 10 200 python tools/kbench.py filter --reps 8 >> gpurun_out/cppipe_kb.log 2>&1 || exit 1
done
echo done
