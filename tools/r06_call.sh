# round 6 working call: GPU tests on the small-workgroup sums default, then its shape sweep
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06j}
V=$PWD/query-compiler-executor_amd/build/var
TESTS="tests/test_gpu_bucket_join.py tests/test_gpu_comm.py tests/test_gpu_fullsize.py tests/test_gpu_primitives.py tests/test_gpu_skew.py" \
REPS=2 bash tools/gpu_ab.sh $T c3 "nt256u4:QE_NOTHING=1" "old:QE_HJ_SUMS_SMALL=0" "nt256u8:QE_LIB_PATH=$V/libqe_nt256u8.so" "nt128u4:QE_LIB_PATH=$V/libqe_nt128u4.so" "nt512u4:QE_LIB_PATH=$V/libqe_nt512u4.so" || exit 1
echo all-done
