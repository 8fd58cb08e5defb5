#!/bin/bash
# On the GPU box: bench line, rocprofv3 kernel trace + stats of bench.py, and
# the PMC passes (separate runs, --kernel-trace only, as the microarch guide
# prescribes) of tools/ba_once.py (cfg4, 20 fixed LM iterations = bench's
# timed region).  Output under gpurun_out/$1.  Every step is time-limited
# and the chain stops at the first failure.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kernel_trace -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$tag -o run -- python tools/ba_once.py cfg4 20 > $OUT/pmc_$tag.log 2>&1
done
echo DONE
