set -o pipefail
mkdir -p gpurun_out
export QE_LIB_PATH=$PWD/query-compiler-executor_amd/build/ab/libqe_STAMPS.so
timeout -k 10 600 bash tools/stamps_c3.sh r05d || exit 1
QE_LIB_PATH=$PWD/query-compiler-executor_amd/build/ab/libqe_STAMPS.so timeout -k 10 120 python tools/stamps.py --what hj > gpurun_out/r05d_hj_stamps.log 2>&1 || exit 1
echo all-done
