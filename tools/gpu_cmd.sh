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
TAILN=3 step t1 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
TAILN=2 step sm 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step bench 300 python bench.py --no-cpu-baseline --no-next-rows --no-end-to-end --no-shard-local
