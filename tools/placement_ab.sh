#!/bin/bash
# Same-box A/B of the C3 line: plain vs under rocprofv3 --kernel-trace, and block placement offsets
# (QE_ALLOC_PAD) -- VERDICT r4 item 1.  Output: gpurun_out/TAG_placement.log
#   tools/placement_ab.sh TAG
set -o pipefail
T=$1
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
L=$O/${T}_placement.log
: > $L
A="--no-cpu --no-faithful --steps 10 --warmup 2"
summ() {   # the bench line's stage table (last JSON line of $1)
  python3 -c "
import json,sys
d=json.loads([l for l in open('$1') if l.startswith('{')][-1])
s=d['stages']; r=d['roofline']
print(d['ms_per_step'], d['kernel_ms_per_step'], d['parity'], 'carry/launch', r['avg_launch_ms'], r['frac'], {k: v['ms_per_step'] for k, v in s.items()})"
}
run_plain() {   # label, env...
  local lab=$1; shift
  echo "== $lab (plain) $*" >> $L
  env "$@" timeout -k 10 240 python3 bench.py $A > $O/${T}_run.json 2> $O/${T}_run.err || { tail -5 $O/${T}_run.err >> $L; return 1; }
  grep "qe sort_pass_carry\|qe alloc" $O/${T}_run.err | head -40 >> $L
  summ $O/${T}_run.json >> $L
}
run_prof() {
  local lab=$1; shift
  echo "== $lab (rocprofv3 --kernel-trace) $*" >> $L
  ( for kv in "$@"; do export "$kv"; done
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_tr -o run -- python3 $R/bench.py $A \
      > $O/${T}_run.json 2> $O/${T}_run.err ) || { tail -5 $O/${T}_run.err >> $L; return 1; }
  grep "qe sort_pass_carry\|qe alloc" $O/${T}_run.err | head -40 >> $L
  summ $O/${T}_run.json >> $L
  rm -rf $O/${T}_tr
}
run_plain base QE_ALLOC_LOG=1 || exit 1
run_prof base QE_ALLOC_LOG=1 || exit 1
for pad in 4096 65536 1048576 2101248; do
  run_plain pad$pad QE_ALLOC_PAD=$pad || exit 1
done
run_plain base2 QE_X=0 || exit 1
run_prof base2 QE_X=0 || exit 1
for pad in 4096 65536 1048576 2101248; do
  run_plain pad${pad}b QE_ALLOC_PAD=$pad || exit 1
done
echo placement-done >> $L
