# same-box A/B: pipelined key gather (default) vs QE_GATHER_PIPE=0, and 8-wide checksums (ck8),
# on the C3 bench line; then the sort/join GPU tests with the default build
set -o pipefail
mkdir -p gpurun_out
D=query-compiler-executor_amd/build/diag
( for L in "" $D/libqe_gp0.so $D/libqe_ck8.so "" $D/libqe_gp0.so $D/libqe_ck8.so; do echo "== ${L:-default}"; QE_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], 'gather_keys', s['gather_keys'], 'checksum', s['checksum'])" || exit 1; done ) > gpurun_out/ab_gck.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sort or gather or checksum or plan or carry" > gpurun_out/ab_gck_tests.log 2>&1
echo rc=$?
