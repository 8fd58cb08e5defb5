# GPU session: -m gpu suite, RANSAC drop-in vs the round-4 build (abso/head), smoke, bench.
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
: > gpurun_out/rab.txt
for r in 1 2; do for d in abso/head structure-from-motion-_amd; do
  timeout -k 10 120 python tools/ransac_ab.py $d 1 >> gpurun_out/rab.txt 2>&1 || { echo "rab $d failed"; exit 1; }
done; done
grep -E "package|dropin|oneshot_score|call_kernels|call " gpurun_out/rab.txt | sed 's#.*/repo/##'
TAILN=2 step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 400 python bench.py
