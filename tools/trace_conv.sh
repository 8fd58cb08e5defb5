#!/bin/bash
# On the GPU box: kernel trace (timestamps) of one warm converged cfg4 solve,
# for tools/trace_gaps.py.  Output under gpurun_out/$1.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python tools/ba_once.py cfg4 50 conv > $OUT/conv.log 2>&1
echo DONE
