set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_comm.py -k "golden" > gpurun_out/r03e_tests.log 2>&1 && \
bash tools/gpu_lib_ab.sh r03uscan2 "us1024:QE_PLAN_USCAN=1" "ordered:QE_PLAN_USCAN=0" "us512:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_US512.so" "us256:QE_LIB_PATH=query-compiler-executor_amd/build/diag/libqe_US256.so"
