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
L=structure-from-motion-_amd/libsfmcore.so
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-next-rows --no-end-to-end --no-shard-local"
TAILN=2 step t1 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "ba_cfg or camera_lds or multi_rank"
for v in a b a b; do
  cp abso/$v.so $L
  TAILN=0 step v$v 200 $B
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/v{sys.argv[1]}.txt").read().strip().splitlines()[-1])
k=d["kernels_ms_per_iter"]; c=d["cfg4"]; k4=c["kernels_ms_per_iter"]
print(sys.argv[1], "cfg5", d["value"], k["backsub_trial"]["ms"], "cfg4", c["value"], k4["backsub_trial"]["ms"])
PY
done
