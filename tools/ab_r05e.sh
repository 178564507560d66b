set -o pipefail
mkdir -p gpurun_out
AB=$PWD/query-compiler-executor_amd/build/ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py tests/test_gpu_local_ranks.py tests/test_gpu_comm.py > gpurun_out/r05e_tests.log 2>&1 || exit 1
# paired first-pass tiles (QE_P1_TM=2): parity first
QE_LIB_PATH=$AB/libqe_tm2.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_bucket_join.py > gpurun_out/r05e_tm2_tests.log 2>&1 || exit 1
REPS=3 bash tools/gpu_lib_ab.sh r05e_c3 "prev:QE_LIB_PATH=$AB/libqe_PREV.so" "late:QE_LIB_PATH=$AB/libqe_late.so" "tm2:QE_LIB_PATH=$AB/libqe_tm2.so" "new:QE_NOTHING=1" || exit 1
( for lib in STAMPS tm2stamps STAMPSLIN; do
    for sel in p1:1 p2:1 p1:4 p2:4; do
      echo "=== $lib $sel"
      w=c3p1; [ "${sel%%:*}" = p2 ] && w=c3p2
      QE_LIB_PATH=$AB/libqe_$lib.so QE_STAMP_SEL=$sel timeout -k 10 120 python tools/stamps.py --what $w 2>&1 | grep -v "^\[stamps\]" || exit 1
    done
  done ) > gpurun_out/r05e_stamps.log 2>&1 || exit 1
QE_LIB_PATH=$AB/libqe_STAMPS.so timeout -k 10 120 python tools/stamps.py --what hj > gpurun_out/r05e_hj_stamps.log 2>&1 || exit 1
echo all-done
