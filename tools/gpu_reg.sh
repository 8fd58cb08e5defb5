set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or smoke or homography" > gpurun_out/rtests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/rtests.txt
[ $rc -eq 0 ] || exit 1
: > gpurun_out/rab.txt
for d in structure-from-motion-_amd abso/u2tree; do
  timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rab.txt 2>&1 || { echo "fail $d"; exit 1; }
done
grep -E "package|dropin|oneshot_score|call_kernels" gpurun_out/rab.txt | sed 's#.*/repo/##'
bash tools/trace_ransac2.sh rtl8 - "SFM_RANSAC_FUSED=0"
