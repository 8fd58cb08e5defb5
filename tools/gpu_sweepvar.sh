set -o pipefail
for n in 1 4; do
  for E in "X=0" "SFM_SWEEP_RANGES=1" "SFM_SWEEP_RANGES=2" "SFM_SWEEP_RANGES=4" "SFM_SWEEP_RANGES=8" "SFM_SWEEP_RANGES=16"; do
    r=$(env $E SFM_SWEEP_VERBOSE=1 timeout -k 10 120 python tools/shard_prof.py $n 20 2>&1 | grep -E "sweep plan|schur" | cut -c1-100 | tr "\n" " ") || exit 1
    echo "N=$n $E $r"
  done
done
