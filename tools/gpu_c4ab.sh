# C4 batch: pipelined compaction on / off, same box
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  QE_CP_PIPE=$v timeout -k 10 300 python bench.py --workload c4 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('QE_CP_PIPE=$v', d['value'], d['ms_per_step'])" >> gpurun_out/c4ab.log || exit 1
done
echo done
