set -o pipefail
for r in 1 2; do for d in - abso/o5 abso/o3; do timeout -k 10 60 python tools/score_sizes.py $d || exit 1; done; done
