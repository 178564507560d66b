# calibration: copy / run-scatter ceilings, pass-1 tile phase stamps, and the current C3 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./build/membench > gpurun_out/ps_membench.log 2>&1 || exit 1
QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_STAMPS.so timeout -k 10 200 python tools/stamps.py --what sort > gpurun_out/ps_stamps.log 2>&1 || exit 1
QE_PROF_SPLIT=1 timeout -k 10 200 python tools/kbench.py sort --reps 6 > gpurun_out/ps_kb.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/ps_bench.json 2> gpurun_out/ps_bench.err || exit 1
echo done
