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
for r in 1 2; do
for tg in 128:2 256:2 128:1 256:1 128:4; do
  T=${tg%:*}; G=${tg#*:}
  SFM_BACKSUB_THREADS=$T SFM_BACKSUB_LANES=$G TAILN=0 step b${T}_$G 200 $B
  python - "b${T}_$G" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/{sys.argv[1]}.txt").read().strip().splitlines()[-1])
print(sys.argv[1], "cfg5", d["value"], d["kernels_ms_per_iter"]["backsub_trial"]["ms"], "cfg4", d["cfg4"]["value"], d["cfg4"]["kernels_ms_per_iter"]["backsub_trial"]["ms"])
PY
done
done
