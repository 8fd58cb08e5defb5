#!/bin/bash
# On the GPU box: kernel + memory-copy timeline of the cfg2 RANSAC drop-in call.
set -e
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 100 python tools/ransac_once.py > $OUT/plain.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o run -- python tools/ransac_once.py > $OUT/trace.log 2>&1
echo DONE
