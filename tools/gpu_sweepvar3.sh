set -o pipefail
for n in 1 8; do
  for E in "X=0" "SFM_SWEEP_RANGES=4 SFM_SWEEP_CHUNK=20000" "SFM_SWEEP_RANGES=2 SFM_SWEEP_CHUNK=20000" "SFM_SWEEP_RANGES=4 SFM_SWEEP_CHUNK=28000" "SFM_SWEEP_RANGES=8 SFM_SWEEP_CHUNK=20000"; do
    r=$(env $E SFM_SWEEP_VERBOSE=1 timeout -k 10 120 python tools/shard_prof.py $n 20 2>&1 | grep -E "sweep plan|schur" | sed 's/chunk trips.*{/{/' | cut -c1-200 | tr "\n" " ") || exit 1
    echo "N=$n $E $r"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/pmc3/p1 -o pmc --output-format csv -- python3 tools/score_once.py > gpurun_out/pmc3/p1.log 2>&1 || echo "pmc failed"
echo PMCDONE
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "queue_overflow or prefilter or ransac_cfg2" > gpurun_out/qtests.txt 2>&1; echo "qtests rc=$?"; tail -3 gpurun_out/qtests.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests -m gpu -k "device_plan" > gpurun_out/ptests.txt 2>&1; echo "ptests rc=$?"; tail -3 gpurun_out/ptests.txt
