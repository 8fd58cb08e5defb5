# GPU session script: each step under its own time limit; a step that ends by
# a signal, a time limit or an abort (rc >= 124) ends the session there.
set -o pipefail
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.txt" | tail -${TAILN:-8}
    if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-next-rows --no-end-to-end --no-shard-local"
TAILN=30 step t1 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "ba_cfg or multi_rank or backsub or perform_bundle"
for v in 0 1 0 1; do
  SFM_BACKSUB_CAM_LDS=$v TAILN=1 step b$v 200 $B
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b{sys.argv[1]}.txt").read().strip().splitlines()[-1])
k=d.get("kernels_ms_per_iter",{}); s=d.get("secondary",{}) or {}
print("LDS", sys.argv[1], d["value"], d["ms_per_step"], {a: k[a] for a in k if "trial" in a or "back" in a})
PY
done
