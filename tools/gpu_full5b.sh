set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/full_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/full_tests.txt
[ $rc -eq 0 ] || exit 1
bash tools/profile_round.sh r5prof2
