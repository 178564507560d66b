# The box state the C3 line runs in: a read-only rocm-smi snapshot (power cap, perf level, VBIOS,
# product), then the C3 query looped ~5 s twice while rocm-smi samples sclk / mclk / power / junction
# temperature continuously beside it -> gpurun_out/TAG_clocks.log; the RESULT lines carry the line's
# ms per query and the sort passes' time, so slow and fast boxes can be told apart by their clocks.
#   tools/clock_probe.sh TAG [STEPS]
set -o pipefail
mkdir -p gpurun_out
T=${1:-clk}; S=${2:-400}
O=gpurun_out/${T}_clocks.log
{ echo "== box"; rocm-smi --showmaxpower --showperflevel --showvbios --showproductname --showdriverversion 2>/dev/null | grep -vE "^=+|^$"; } > $O
( while true; do echo "t=$(date +%s.%N | cut -c1-14)"; rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|fclk|Package Power|junction"; done ) >> $O 2>&1 &
SMI=$!
trap 'kill $SMI 2>/dev/null' EXIT
for rep in 1 2; do
  echo "== run $rep start $(date +%s.%N | cut -c1-14)" >> $O
  timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps $S --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print('RESULT', d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in list(s.items())[:4]})" >> $O 2>&1 || exit 1
  echo "== run $rep end $(date +%s.%N | cut -c1-14)" >> $O
done
echo all-done
