# sort_pass_carry's spread across runs on one box: the GPU's clocks, power and temperature sampled
# (read-only rocm-smi) while the C3 line runs three times back to back -> gpurun_out/TAG_clocks.log
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05zb}
O=gpurun_out/${T}_clocks.log
: > $O
for rep in 1 2 3; do
  ( for i in $(seq 120); do echo "t=$(date +%s.%N | cut -c1-14) rep=$rep"; rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|fclk|Power|Temperature" ; sleep 0.5; done ) >> $O 2>&1 &
  smi=$!
  echo "== run $rep" >> $O
  timeout -k 10 240 python bench.py --no-cpu --no-faithful --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['stages']; print('RESULT', d['ms_per_step'], d['kernel_ms_per_step'], {k: v['ms_per_step'] for k, v in list(s.items())[:4]})" >> $O 2>&1
  rc=$?
  kill $smi 2>/dev/null; wait $smi 2>/dev/null
  [ $rc -eq 0 ] || exit 1
done
echo all-done
