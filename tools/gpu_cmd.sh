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
TAILN=4 step t1 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
TAILN=2 step sm 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=0 step bench 600 python bench.py
python - <<'PY'
import json
d=json.loads(open("gpurun_out/bench.txt").read().strip().splitlines()[-1])
print("cfg5", d["value"], d["ms_per_step"], d["converged_LM_it_per_s"], d["roofline"]["frac"])
c=d["cfg4"]; print("cfg4", c["value"], c["ms_per_step"], c["converged_LM_it_per_s"])
PY
