# GPU session: -m gpu suite, the RANSAC prefilter A/B, bench, create/obs phases.
set -o pipefail
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.txt" | tail -${TAILN:-4}
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
TAILN=3 step tests 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu
TAILN=12 step rab 300 python tools/ransac_ab.py
TAILN=2 step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 400 python bench.py
TAILN=4 step create5 200 python tools/create_once.py cfg5
TAILN=4 step create4 200 python tools/create_once.py cfg4
TAILN=8 step obs5 300 python tools/obs_probe.py cfg5
