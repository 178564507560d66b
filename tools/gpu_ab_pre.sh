# same-box A/B of the lookback-free two-level sort on the C3 bench line and the sort alone
set -o pipefail
mkdir -p gpurun_out
( for v in 1 0 1 0; do echo "== PRE=$v"; QE_PROF_SPLIT=1 QE_SORT_PRE=$v timeout -k 10 200 python tools/kbench.py sort --reps 8 || exit 1; done ) > gpurun_out/kb_sortpre.log 2>&1 && \
( for v in 1 0 1 0; do echo "== PRE=$v"; QE_SORT_PRE=$v timeout -k 10 240 python bench.py --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'])" || exit 1; done ) > gpurun_out/ab_pre.log 2>&1
echo rc=$?
