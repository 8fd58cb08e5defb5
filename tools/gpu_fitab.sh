set -o pipefail
for r in 1 2 3; do for d in - abso/oldfit; do echo "$d $(timeout -k 10 120 python tools/dropin_phases.py $d)"; done; done
bash tools/trace_ransac2.sh rtl12 -
