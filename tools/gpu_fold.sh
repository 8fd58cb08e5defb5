set -o pipefail
for r in 1 2; do for E in "SFM_GJR_FOLD=0" "SFM_GJR_FOLD=1"; do
  for n in 1 8; do echo "$E N=$n $(env $E timeout -k 10 120 python tools/shard_prof.py $n 20 2>&1 | tail -1)"; done
done; done
