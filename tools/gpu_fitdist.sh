set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or smoke or homography or f8" > gpurun_out/ftests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ftests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for d in - abso/oldfit; do timeout -k 10 60 python tools/fit_sizes.py $d || exit 1; done; done
for r in 1 2; do echo "tree $(timeout -k 10 120 python tools/dropin_phases.py)"; done
