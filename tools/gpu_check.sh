#!/bin/bash
# Dev helper: rebuild in-tree (fail loudly), then run the GPU parity tests,
# the BA/RANSAC probe and (optionally) a rocprofv3 kernel trace of bench.py
# on one MI355X through gpurun.  Usage: tools/gpu_check.sh [prof_tag]
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C structure-from-motion-_amd
make -s -C oracle
TAG=${1:-}
# steps chained with && so nothing else touches the GPU after a failure
CMD='timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && timeout -k 10 300 python tools/probe_ba.py > gpurun_out/probe.log 2>&1'
if [ -n "$TAG" ]; then
  CMD="$CMD && cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1"
fi
timeout 1700 /usr/local/graft/bin/gpurun --timeout 1000 -- "$CMD" 2>&1 | tail -1
rm -f gpurun_out/probe.log.stale; tail -2 gpurun_out/gpu_tests.log
grep -E "cfg|fixed|EXIT|Err" gpurun_out/probe.log || true
if [ -n "$TAG" ]; then
python3 - "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/{sys.argv[1]}/run_kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:18]:
    print(f"{r['Name'][:50]:50s} calls={r['Calls']:>6} avg_us={float(r['AverageNs'])/1e3:9.2f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f} pct={float(r['Percentage']):.1f}")
PY
fi
