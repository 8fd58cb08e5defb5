"""cfg2 F-RANSAC drop-in calls (in-call sampling) for a rocprofv3 timeline:
3 warm calls, then 5; prints each call's wall time."""
import os, random, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "structure-from-motion-_amd")]
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402
x1, x2, _, _ = syn.two_view(n=5000, seed=0)
for i in range(8):
    random.seed(0)
    t = time.perf_counter()
    core.ransac_f8_pyrandom(x1, x2, 16384, 0.06)
    print(i, round((time.perf_counter() - t) * 1e3, 3), "ms", [round(v, 4) for v in core.last_timings()], flush=True)
