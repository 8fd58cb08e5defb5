#!/bin/bash
# per-point lane-group sizes of k_backsub_trial / k_linearize and backsub grid (cfg4 fixed10 timings)
set -e
for BL in 1 2 4 8; do
  echo "BACKSUB_LANES=$BL $(SFM_BACKSUB_LANES=$BL timeout -k 10 100 python tools/probe_ba.py 2>&1 | grep -A2 '^cfg4' | grep fixed10 | grep -o "'backsub_trial': [0-9.]*")"
done
for BB in 512 1024 2048; do
  echo "BACKSUB_BLOCKS=$BB $(SFM_BACKSUB_BLOCKS=$BB timeout -k 10 100 python tools/probe_ba.py 2>&1 | grep -A2 '^cfg4' | grep fixed10 | grep -o "'backsub_trial': [0-9.]*")"
done
for LL in 2 4 8; do
  echo "LINEARIZE_LANES=$LL $(SFM_LINEARIZE_LANES=$LL timeout -k 10 100 python tools/probe_ba.py 2>&1 | grep -A2 '^cfg4' | grep fixed10 | grep -o "'linearize': [0-9.]*")"
done
