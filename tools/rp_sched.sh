#!/bin/bash
# In-call RANSAC wall time (tools/ransac_once.py, last 3 calls) per chunk schedule
set -e
for S in "" "1024,4096" "512,1024,1536,2048,3072,4096" "1024,1024,2048,2048,4096" "512,1024,2048,4096" "768,1536,3072,4096" "1024,2048,3072,4096,6144" "512,1024,1536,2048,3072,4096,4096,512"; do
  echo "== schedule '$S'"
  SFM_RP_SCHEDULE="$S" SFM_HOSTPROF=1 timeout -k 10 60 python tools/ransac_once.py 2>&1 | tail -4 | grep -v "^hostprof" | cut -c1-16
done
