#!/bin/bash
# same-box A/B of library builds / env knobs on the C5 line (two rounds each):
#   tools/gpu_c5_ab.sh TAG "LABEL:ENV..." ...   -> gpurun_out/TAG_c5.log
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
( for rep in 1 2; do for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    echo "== $label"
    env $envs timeout -k 10 300 python bench.py --workload c5 --no-cpu --steps 5 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'], {k: v['ms_per_step'] for k, v in d['stages'].items()})" || exit 1
  done; done ) > gpurun_out/${T}_c5.log 2>&1
rc=$?; echo c5ab rc=$rc; exit $rc
