# GPU session script: each step under its own time limit; a step that ends by
# a signal, a time limit or an abort (rc >= 124) ends the session there.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.txt" | tail -${TAILN:-8}
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-next-rows --no-end-to-end --no-shard-local"
TAILN=4 step t1 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "ba or reduced or schur or gj or perform_bundle"
rm -rf gpurun_out/ks
TAILN=0 step ks 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o ks --output-format csv -- python3 tools/ba_once.py cfg5
f=$(find gpurun_out/ks -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"])/1000,2))
PY
for i in 1 2; do
TAILN=0 step b$i 200 $B
python - $i <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b{sys.argv[1]}.txt").read().strip().splitlines()[-1])
print("cfg5", d["value"], d["ms_per_step"], d["converged_LM_it_per_s"], {k: v["ms"] for k, v in d["kernels_ms_per_iter"].items()})
c=d["cfg4"]; print("cfg4", c["value"], c["ms_per_step"], c["converged_LM_it_per_s"], {k: v["ms"] for k, v in c["kernels_ms_per_iter"].items()})
PY
done
