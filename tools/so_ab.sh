#!/bin/bash
# A/B two builds of libsfmcore.so (abso/a.so, abso/b.so) on one box: probe_ransac, alternated
set -e
L=structure-from-motion-_amd/libsfmcore.so
for V in a b a b; do
  cp abso/$V.so $L
  echo "== $V"
  timeout -k 10 100 python tools/probe_ransac.py 2>&1 | head -4
done
