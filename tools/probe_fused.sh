#!/bin/bash
# A/B of the sweep-fused camera blocks: converged + fixed cfg4 solves (probe_ba.py)
set -e
SFM_CAMLIN_FUSED=0 timeout -k 10 120 python tools/probe_ba.py > gpurun_out/probe_unfused.log 2>&1
SFM_CAMLIN_FUSED=1 timeout -k 10 120 python tools/probe_ba.py > gpurun_out/probe_fused.log 2>&1
echo DONE
