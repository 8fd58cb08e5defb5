"""Host phases of the cfg2 F-RANSAC drop-in call (sfm_ransac_f8_dropin's
stamps, sfm_last_timings [6..10]) beside the Python wall times: medians of
30 calls.  Call timing off (no HIP events), as the drop-in runs."""
import os, random, statistics as st, sys, time
_here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_here, "structure-from-motion-_amd")]
if len(sys.argv) > 1 and sys.argv[1] != "-":
    sys.path.insert(0, os.path.abspath(sys.argv[1]))
import numpy as np  # noqa: E402
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402
from GetInliersRANSAC import GetInliersRANSAC  # noqa: E402
x1, x2, _, _ = syn.two_view(n=5000, seed=0)
idx = np.arange(5000)
rows = {k: [] for k in ("draw", "pre", "enqueued", "drained", "c_return", "lib_call", "dropin")}
for i in range(40):
    random.seed(0)
    t = time.perf_counter()
    core.ransac_f8_dropin(x1, x2, 16384, 0.06)
    lib = (time.perf_counter() - t) * 1e3
    tm = core.last_timings()
    random.seed(0)
    t = time.perf_counter()
    GetInliersRANSAC(x1, x2, idx, 0.06, 16384)
    d = (time.perf_counter() - t) * 1e3
    if i >= 10:
        for k, v in zip(("draw", "pre", "enqueued", "drained", "c_return"), tm[6:11]):
            rows[k].append(v)
        rows["lib_call"].append(lib)
        rows["dropin"].append(d)
print(" ".join(f"{k}={st.median(v):.4f}" for k, v in rows.items()))
