# A/B of the aggregate join's tile kernel (C5 bench agg_count): default, no walks, one walk, tile shapes
set -o pipefail
mkdir -p gpurun_out
for v in default ag512x8 ag256x8; do
  if [ $v = default ]; then L=""; else L=query-compiler-executor_amd/build/diag/libqe_$v.so; fi
  echo "== $v" >> gpurun_out/agab.log
  QE_LIB_PATH=$L timeout -k 10 200 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['stages']))" >> gpurun_out/agab.log || exit 1
done
echo done
