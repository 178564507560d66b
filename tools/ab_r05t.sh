# r05t: the hash join restricted to joins whose sides are both small (C4 A/B: both < 2^20, both < 2^22, off)
timeout -k 10 700 bash tools/gpu_c4_ab.sh r05t "h20:QE_NOTHING=1" "h22:QE_HASH_JOIN=22" "merge:QE_HASH_JOIN=0" || exit 1
