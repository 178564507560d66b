# host-gap change (deferred largest-bucket checks) + compact-kernel phase stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bucket_join.py tests/test_gpu_comm.py > gpurun_out/gap_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/gap_bench.json 2> gpurun_out/gap_bench.err || exit 1
for v in stamps:8192 stamps12:12288; do
  QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_${v%%:*}.so timeout -k 10 120 python tools/stamps.py --what cp --cp-tile ${v##*:} >> gpurun_out/gap_stamps.log 2>&1 || exit 1
done
echo done
