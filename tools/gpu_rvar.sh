# GPU session: RANSAC score variants (abso/*) alternated, the tree's GPU tests, bench.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/rvar.txt
for r in 1 2; do
  for d in abso/head structure-from-motion-_amd abso/v4f6 abso/v4f5 abso/v4f4; do
    timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rvar.txt 2>&1 || { echo "fail $d"; exit 1; }
  done
done
grep -E "package|dropin|oneshot_score|call_kernels" gpurun_out/rvar.txt | sed 's#.*/repo/##'
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/tests.txt 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/tests.txt
