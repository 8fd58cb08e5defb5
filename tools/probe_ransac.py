"""Dev probe: where the end-to-end time of the in-call-sampling RANSAC goes
(host draw, GPU span, Python wrapper) on the cfg2 two-view problem."""
import os
import random
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "structure-from-motion-_amd")]
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

x1, x2, _, _ = syn.two_view(n=5000, outlier_frac=0.4, seed=2)
H = int(os.environ.get("H", 16384))
core.set_call_timing(True)  # device split of the in-call path
for fn in (core.ransac_f8_pyrandom, core.ransac_h4_pyrandom):
    for _ in range(3):
        random.seed(0)
        fn(x1, x2, H, 0.06)
    w = []
    tm = []
    for _ in range(20):
        random.seed(0)
        t = time.perf_counter()
        fn(x1, x2, H, 0.06)
        w.append((time.perf_counter() - t) * 1e3)
        tm.append(core.last_timings())
    tm = np.median(np.array(tm), axis=0)
    print(fn.__name__, "wall ms %.3f" % np.median(w), "timings", np.round(tm, 4).tolist())
# Python glue alone: the MT state round trip the drop-in does per call
t = time.perf_counter()
for _ in range(200):
    v, st, g = core._mt_state()
    core._mt_restore(v, st, g)
print("mt state round trip ms %.4f" % ((time.perf_counter() - t) / 200 * 1e3))
# kernel split of the given-table path (upload, kernels, download, score, fit, select)
random.seed(0)
tbl = core.sample_table(len(x1), 8, H)
for _ in range(3):
    core.ransac_f8(x1, x2, tbl, 0.06)
tm = []
for _ in range(20):
    core.ransac_f8(x1, x2, tbl, 0.06)
    tm.append(core.last_timings())
print("table path ms (up, kernels, down, score, fit, select)", np.round(np.median(np.array(tm), axis=0), 4).tolist())
for h in (512, 2048, 4096):
    t4 = []
    for _ in range(10):
        core.ransac_f8(x1, x2, tbl[:h], 0.06)
        t4.append(core.last_timings()[4])
    print("fit ms at H=%d: %.4f" % (h, np.median(t4)))
