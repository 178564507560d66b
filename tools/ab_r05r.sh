set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
REPS=3 bash tools/gpu_lib_ab.sh r05r_c3 "new:QE_NOTHING=1" "tmnone:QE_LIB_PATH=$AB/libqe_tmnone.so" "rwch16:QE_LIB_PATH=$AB/libqe_rwch16.so" "rwch4:QE_LIB_PATH=$AB/libqe_rwch4.so" || exit 1
echo all-done
