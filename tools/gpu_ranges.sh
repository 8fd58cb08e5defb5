set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "ba or plan or reduced or multi_rank or bundle or smoke" > gpurun_out/btests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/btests.txt
[ $rc -eq 0 ] || exit 1
for n in 1 2 8; do echo "N=$n $(timeout -k 10 120 python tools/shard_prof.py $n 20 2>&1 | tail -1)"; done
timeout -k 10 600 python bench.py --no-cpu-baseline --no-next-rows > gpurun_out/bench_rng.json 2> gpurun_out/bench_rng.err; echo "bench rc=$?"
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_rng.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['cfg4']['value'], d['converged_LM_it_per_s'], d['ransac']['hyps_per_s_end_to_end'], json.dumps(d['end_to_end']['phases_ms']), json.dumps(d['cfg4']['end_to_end']['phases_ms']))"
