# r05x: the chain bucket join in its loop form with one block per bucket (the default after r05w) against the previous commit
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
REPS=3 timeout -k 10 700 bash tools/gpu_lib_ab.sh r05x_c3 "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05x "new:QE_NOTHING=1" "prev:QE_LIB_PATH=$AB/libqe_PREV.so" || exit 1
echo all-done
