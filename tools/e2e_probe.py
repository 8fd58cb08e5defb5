"""Dev probe (round 4): the BA drop-in's whole call (perform_bundle_adjustment
on dense matrices, to convergence) at cfg4 / cfg5, twice, with the phase split
(BundleAdjustment.last_timings) and, with SFM_CREATE_TIMING=1, sfm_ba_create's
host phases on stderr.  Usage: e2e_probe.py [cfg5]"""
import os, sys, time, json, contextlib, io
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
sys.path.insert(0, R)
import numpy as np
import bench
print(json.dumps(bench.end_to_end_ba(sys.argv[1] if len(sys.argv) > 1 else "cfg5"), indent=1))
