# GPU session: -m gpu suite, RANSAC A/B vs round 4, a timing-off BA kernel trace (gaps).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/tests.txt; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/rab.txt
for r in 1 2; do for d in abso/head structure-from-motion-_amd; do
  timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rab.txt 2>&1 || { echo "rab $d failed"; exit 1; }
done; done
grep -E "package|dropin|oneshot_score|call_kernels|call " gpurun_out/rab.txt | sed 's#.*/repo/##'
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/cfg5 -o kt -- python3 tools/ba_once.py cfg5 20 > gpurun_out/gap/cfg5.log 2>&1 || { echo "trace failed"; exit 1; }
head -1 gpurun_out/gap/cfg5.log
echo done
