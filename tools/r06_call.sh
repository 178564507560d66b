# round 6 working call: C4 knobs on this round's build (longest-first lane order, scan keys, sums form)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r06o}
bash tools/gpu_ab.sh $T c4 "base:QE_NOTHING=1" "inorder:QE_LANE_ORDER=0" "gatherkeys:QE_SCAN_KEYS=0" "oldsums:QE_HJ_SUMS_SMALL=0" || exit 1
echo all-done
