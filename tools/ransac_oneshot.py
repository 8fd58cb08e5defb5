"""The one-shot F-RANSAC launch (core.ransac_f8 on a drawn cfg2 table of
16,384 hypotheses: one fit + one score launch) for rocprofv3 PMC passes --
bench.py's RANSAC roofline reads SQ_INSTS_VALU (and the FP64 splits) of
k_epi_score from them.  3 warm calls, then 5."""
import os
import random
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "structure-from-motion-_amd")]
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

x1, x2, _, _ = syn.two_view(n=5000, seed=0)
random.seed(0)
samples = core.sample_table(len(x1), 8, 16384)
for i in range(8):
    best, F, mask = core.ransac_f8(x1, x2, samples, 0.06)[:3]
print("best", best, "inliers", int(mask.sum()), flush=True)
