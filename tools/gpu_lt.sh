set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or homography or smoke" > gpurun_out/ltests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ltests.txt
