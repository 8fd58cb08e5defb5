#!/bin/bash
# RANSAC in-call chunk schedule sweep (first chunk x ramp x chunk): wall ms per call
set -e
for RAMP in 0 1; do for FIRST in 1024 2048 4096; do for CH in 4096 8192; do
  echo "ramp=$RAMP first=$FIRST chunk=$CH $(SFM_RP_RAMP=$RAMP SFM_RP_FIRST=$FIRST SFM_RP_CHUNK=$CH timeout -k 10 60 python tools/ransac_once.py | tail -6 | awk '{print $2}' | sort -n | head -3 | tr '\n' ' ')"
done; done; done
