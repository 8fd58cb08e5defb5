set -o pipefail
timeout -k 10 800 python bench.py > gpurun_out/bench_final2.json 2> gpurun_out/bench_final2.err; echo "bench rc=$?"
