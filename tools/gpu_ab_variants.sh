# same-box A/B of the default libqe against variant builds on the C3 bench line:
#   bash tools/gpu_ab_variants.sh TAG VARIANT...   (build/diag/libqe_VARIANT.so, tools/build_variant.sh)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
D=query-compiler-executor_amd/build/diag
L=""; for v in "$@"; do L="$L $D/libqe_$v.so"; done
( for r in 1 2; do for lib in "" $L; do echo "== ${lib:-default}"; QE_LIB_PATH=$lib timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in s.items()})" || exit 1; done; done ) > gpurun_out/${T}_ab.log 2>&1
echo rc=$?
