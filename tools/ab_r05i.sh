set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 bash tools/gpu_c4_ab.sh r05i "base:QE_NOTHING=1" "swap4:QE_MJ_SWAP=4" "swap16:QE_MJ_SWAP=16" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
echo all-done
