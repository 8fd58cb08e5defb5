set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/chain_probe > gpurun_out/chain_probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "reduced_solve or gj_solve or cfg4_matches or cfg5_matches or many_cameras or midsize or multi_rank_matches or multi_rank_baseline or device_plan or failure_contract or split_and_gjr" > gpurun_out/solve_tests.txt 2>&1; rc=$?
tail -5 gpurun_out/solve_tests.txt
[ $rc -ne 0 ] && exit $rc
SFM_CREATE_TIMING=1 timeout -k 10 120 python tools/ba_once.py cfg5 2 > gpurun_out/create_cfg5.txt 2>&1
SFM_CREATE_TIMING=1 SFM_PLAN_HOST=1 timeout -k 10 120 python tools/ba_once.py cfg5 2 > gpurun_out/create_cfg5_host.txt 2>&1
timeout -k 10 600 bash tools/ab_pkgs.sh 2 abso/old structure-from-motion-_amd > gpurun_out/ab_solve.txt 2>&1; rc=$?
grep -oE "== .*|cfg[45]: .*cholesky [0-9.]+" gpurun_out/ab_solve.txt | sed -E 's/linearize.*cholesky/... cholesky/'
exit $rc
