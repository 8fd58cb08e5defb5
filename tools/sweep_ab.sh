#!/bin/bash
# A/B of the sweep's group plan: balanced (default) vs power-of-two (SFM_SWEEP_POW2=1), cfg4 and cfg5
set -e
for P in 1 0 1 0; do
  echo "POW2=$P"
  SFM_SWEEP_POW2=$P timeout -k 10 100 python tools/probe_ba.py 2>&1 | grep -A2 "^cfg[45]" | grep fixed10 | cut -c1-120
done
