set -o pipefail
for d in - abso/f1 abso/f2; do timeout -k 10 60 python tools/fit_sizes.py $d || exit 1; done
