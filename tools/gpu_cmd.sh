set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "reduced_solve or gj_solve_matches or cfg4_matches or cfg5_matches" > gpurun_out/t1.log 2>&1; echo "pytest rc=$?"
tail -5 gpurun_out/t1.log
timeout -k 10 120 python -u tools/gjr_timeline.py 300 > gpurun_out/tl300.txt 2>&1 && timeout -k 10 120 python -u tools/gjr_timeline.py 1200 > gpurun_out/tl1200.txt 2>&1; echo "tl rc=$?"
timeout -k 10 300 python -u tools/gj_ab.py SFM_SOLVE gjr,gjseg 2 > gpurun_out/ab1.txt 2>&1; echo "ab rc=$?"
tail -4 gpurun_out/ab1.txt
