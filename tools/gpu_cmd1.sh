set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/bin/chain_probe > gpurun_out/chain_probe.txt 2>&1 || exit 1
bash tools/gpu_cmd.sh
