set -o pipefail
for r in 1 2; do for d in - abso/f3 abso/f4; do timeout -k 10 60 python tools/fit_sizes.py $d || exit 1; done; done
