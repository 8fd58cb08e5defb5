#!/bin/bash
# The one GPU-box entry point for measurements (round 6; replaces the
# round-1..5 one-off gpu_*.sh scripts).  Run it under gpurun from the repo
# root:  gpurun -- 'bash tools/gpu.sh <what> [out]'.  Every GPU step has its
# own time limit and the steps stop at the first failure; output goes under
# gpurun_out/<out> (default: <what>).
#   tests     the -m gpu suite, then smoke()
#   bench     bench.py (N = 1, defaults)
#   solve     the reduced solve's per-pivot timeline (gjr_timeline.py, n = 1200
#             and 300) and the BA kernel split with it and the Cholesky (gj_ab.py)
#   e2e       the drop-in perform_bundle_adjustment at cfg4 and cfg5, with
#             sfm_ba_create's host phases (SFM_CREATE_TIMING=1)
#   profile   tools/profile_round.sh (bench, rocprofv3 kernel stats, PMC passes)
set -o pipefail
W=${1:?what}
OUT=gpurun_out/${2:-$W}
mkdir -p $OUT
case $W in
tests)
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit 1
  tail -3 $OUT/gpu_tests.txt; tail -1 $OUT/smoke.txt ;;
bench)
  timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
  tail -c 600 $OUT/bench.json ;;
solve)
  timeout -k 10 300 python -u tools/gj_ab.py SFM_SOLVE gj,chol 3 > $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python -u tools/gjr_timeline.py 1200 > $OUT/tl1200.txt 2>&1 || exit 1
  timeout -k 10 60 python -u tools/gjr_timeline.py 300 > $OUT/tl300.txt 2>&1 || exit 1
  tail -4 $OUT/ab.txt ;;
e2e)
  for C in cfg4 cfg5; do
    SFM_CREATE_TIMING=1 timeout -k 10 300 python -u tools/e2e_probe.py $C > $OUT/e2e_$C.txt 2>&1 || exit 1
  done ;;
profile)
  bash tools/profile_round.sh ${2:-profile} ;;
*) echo "unknown: $W"; exit 2 ;;
esac
