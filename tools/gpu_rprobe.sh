set -o pipefail
: > gpurun_out/rprobe.txt
for r in 1 2; do for d in structure-from-motion-_amd abso/u2p2 abso/u2p3; do
  timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rprobe.txt 2>&1 || { echo "fail $d"; exit 1; }
done; done
grep -E "package|dropin|oneshot_score|call_kernels" gpurun_out/rprobe.txt | sed 's#.*/repo/abso/##; s#.*/repo/##' | awk '/package/{p=$2} /call_kernels/{ck=$4} /dropin/{d=$4} /oneshot_score/{print p, "call_kernels", ck, "dropin", d, "oneshot", $4}'
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "ransac or smoke" > gpurun_out/rtests.txt 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/rtests.txt
