set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or smoke or homography or pnp" > gpurun_out/rtests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/rtests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for E in "SFM_RANSAC_LAUNCHER=1" "SFM_RANSAC_LAUNCHER=0"; do echo "$E $(env $E timeout -k 10 120 python tools/dropin_phases.py)"; done; done
