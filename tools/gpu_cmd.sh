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
step acc 120 python -u tools/gjr_accuracy.py tools/_abG3
for v in HD G3 HD G3; do
  TAILN=2 step ab$v 300 python -u tools/gj_ab.py SFM_SOLVE gjr 2 tools/_ab$v
done
