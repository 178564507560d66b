# lookback-free two-level sort: its tests, a sort A/B (QE_SORT_PRE=1 vs 0, second pass timed on
# its own), then (FULL=1) the whole GPU suite and the C3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "sort" --timeout 120 --timeout-method thread > gpurun_out/sortpre_tests.log 2>&1 && \
( for v in 1 0 1; do echo "== PRE=$v"; QE_PROF_SPLIT=1 QE_SORT_PRE=$v timeout -k 10 200 python tools/kbench.py sort --reps 8 || exit 1; done ) > gpurun_out/kb_sortpre.log 2>&1 && \
if [ "${FULL:-0}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 240 python bench.py --no-cpu > gpurun_out/bench_c3.log 2>&1
fi
echo rc=$?
