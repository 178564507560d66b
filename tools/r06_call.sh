# round 6 working call: the plan's fused scan at 512 threads a workgroup / 8 steps a wave
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06s}
V=$PWD/query-compiler-executor_amd/build/var
REPS=2 bash tools/gpu_ab.sh $T c3 "base:QE_NOTHING=1" "usb512:QE_LIB_PATH=$V/libqe_usb512.so" "uss8:QE_LIB_PATH=$V/libqe_uss8.so" || exit 1
echo all-done
