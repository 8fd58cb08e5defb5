"""Model of k_backsub_trial's camera reads from LDS (round 6, VERDICT round 5
#4): 64 lanes = 32 points x 2 lanes, lane (point, s) reads observations s,
s + 2, ...; per observation six ds_read_b128 of the camera's 240-B record
(stride 15 x 16 B).  A b128 read is served as four 16-lane passes over 16
positions of 16 B; a pass takes as many cycles as the most distinct
addresses on one position (equal addresses broadcast).  Prints the conflict
cycles per b128 read for the synthetic cfg5 points in their order and
sorted lexicographically by camera tuple.  Usage: lds_conflict_sim.py [cfg5]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "structure-from-motion-_amd"))
import sfm_synthetic as syn  # noqa: E402

p = syn.ba_problem_cfg(sys.argv[1] if len(sys.argv) > 1 else "cfg5", dense=False)
k, npt = p["k"], p["n_pts"]
cams = p["cam_idx"].reshape(npt, k)  # point-major, cameras ascending


def conflicts(cams, G=2, nwaves=4000, stride16=15):
    tot = n = 0
    rng = np.random.default_rng(0)
    for s0 in rng.integers(0, npt // 32 - 1, nwaves) * 32:
        pts = cams[s0:s0 + 32]
        for step in range(k // G):
            c = np.empty(64, dtype=np.int64)
            for s in range(G):
                c[s::G] = pts[:, s + step * G]
            for f in range(6):
                addr = c * stride16 + f  # 16-B units
                pos = addr % 16
                for q in range(4):
                    a, ps = addr[16 * q:16 * q + 16], pos[16 * q:16 * q + 16]
                    tot += max(len(np.unique(a[ps == v])) for v in range(16)) - 1
                n += 1
    return tot / n


print("points in their order:", round(conflicts(cams), 2), "conflict cycles per b128 read")
print("points sorted by camera tuple:", round(conflicts(cams[np.lexsort(cams.T[::-1])]), 2))
