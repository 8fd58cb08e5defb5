set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or smoke" > gpurun_out/rtests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/rtests.txt
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for d in structure-from-motion-_amd abso/prio0; do timeout -k 10 120 python tools/ransac_ab.py $d 1 | grep -E "package|dropin|call_kernels" | sed 's#.*/repo/##'; done; done
bash tools/trace_ransac2.sh rtl10 -
