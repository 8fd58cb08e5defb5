#!/bin/bash
# Kernel timelines of the cfg2 drop-in call under several env settings.
# usage: tools/trace_ransac2.sh TAG "ENV1" "ENV2" ...   (ENV: "A=1 B=2" or "-")
set -e
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for E in "$@"; do
  OUT=gpurun_out/$TAG/v$i; mkdir -p $OUT
  [ "$E" = "-" ] && E=""
  echo "v$i: $E" > $OUT/env.txt
  env $E timeout -k 10 100 python tools/ransac_once.py > $OUT/plain.log 2>&1
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python tools/ransac_once.py > $OUT/trace.log 2>&1
  i=$((i+1))
done
echo DONE
