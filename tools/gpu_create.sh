set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "plan or ba_cfg4 or ba_cfg5 or multi_rank or dense or coo or many_cameras or sweep_split" > gpurun_out/ctests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ctests.txt
[ $rc -eq 0 ] || exit 1
for W in cfg4 cfg5; do
  echo "== $W new"; timeout -k 10 120 python tools/create_once.py $W 2>&1 | grep -E "^create|csr|plan:|chunk" | tail -8
  echo "== $W global"; SFM_CSR_CNT_GLOBAL=1 SFM_PLAN_COUNTS_GLOBAL=1 SFM_PLAN_CHUNK_SPLIT=1 timeout -k 10 120 python tools/create_once.py $W 2>&1 | grep -E "^create" | tail -2
done
