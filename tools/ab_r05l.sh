set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
REPS=3 bash tools/gpu_lib_ab.sh r05l_c3 "new:QE_NOTHING=1" "p2res2:QE_LIB_PATH=$AB/libqe_p2res.so QE_P2_RESIDENT=2" "p2res4:QE_LIB_PATH=$AB/libqe_p2res.so QE_P2_RESIDENT=4" "p2res0:QE_LIB_PATH=$AB/libqe_p2res.so" || exit 1
timeout -k 10 900 bash tools/round_end.sh r05l c4 || exit 1
echo all-done
