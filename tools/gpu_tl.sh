set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/gjr_timeline2.py abso/stamps 1200 > gpurun_out/tl1200.txt 2>&1 || exit 1
timeout -k 10 120 python tools/gjr_timeline2.py abso/stamps 300 > gpurun_out/tl300.txt 2>&1 || exit 1
timeout -k 10 200 python tools/create_once.py cfg5 > gpurun_out/create_once_cfg5.txt 2>&1 || exit 1
timeout -k 10 200 python tools/create_once.py cfg4 > gpurun_out/create_once_cfg4.txt 2>&1 || exit 1
