#!/bin/bash
# A/B of two package builds (dirs holding _sfmcore.py + libsfmcore.so) on one
# box: the BA kernel split at cfg4 / cfg5 (tools/gj_ab.py, 20 fixed LM
# iterations), alternated, each run in its own process.  Usage:
#   tools/ab_pkgs.sh ROUNDS DIR_A DIR_B
R=$1; A=$2; B=$3
for i in $(seq 1 $R); do
  for D in $A $B; do
    echo "== $D"
    timeout -k 10 200 python tools/gj_ab.py SFM_AB_DUMMY 0 1 $D 2>&1 | grep -E "^round" || exit 1
  done
done
