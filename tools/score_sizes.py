"""The cfg2 one-shot F score (given table, HIP events) at several hypothesis
counts: median ms of 20 calls each.  Env SFM_EPI_* knobs apply."""
import os, random, statistics as st, sys
_here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_here, "structure-from-motion-_amd")]
if len(sys.argv) > 1 and sys.argv[1] != "-":
    sys.path.insert(0, os.path.abspath(sys.argv[1]))
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402
x1, x2, _, _ = syn.two_view(n=5000, seed=0)
random.seed(0)
table = core.sample_table(5000, 8, 16384)
core.set_call_timing(True)
out = []
for H in (1024, 3072, 4096, 8192, 16384):
    v = []
    for _ in range(20):
        core.ransac_f8(x1, x2, table[:H], 0.06)
        v.append(core.last_timings()[3])
    out.append(f"H={H}:{st.median(v[5:]) * 1e3:.1f}us")
print(sys.argv[1] if len(sys.argv) > 1 else "", os.environ.get("TAG", ""), " ".join(out), flush=True)
