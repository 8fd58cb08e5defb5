#!/bin/bash
# Same-box A/B of the fused next-chunk fit (abso/w{5,6,8}.so = occupancy cap
# of the fused score launch) against fit-then-score (SFM_RANSAC_FUSED=0).
set -e
L=structure-from-motion-_amd/libsfmcore.so
for R in 1 2; do
  for V in w8:0 w8:1 w6:1 w5:1; do
    cp abso/${V%:*}.so $L
    echo "== ${V%:*} fused=${V#*:}"
    SFM_RANSAC_FUSED=${V#*:} timeout -k 10 100 python tools/probe_ransac.py 2>&1 | head -2
  done
done
