"""cfg2 one-shot F scores (given table) for rocprofv3 counter passes:
python tools/score_once.py [PKGDIR]"""
import os
import random
import sys

_here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_here, "structure-from-motion-_amd")]
if len(sys.argv) > 1:
    sys.path.insert(0, os.path.abspath(sys.argv[1]))
import _sfmcore as core  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

x1, x2, _, _ = syn.two_view(n=5000, seed=0)
random.seed(0)
table = core.sample_table(5000, 8, 16384)
for _ in range(5):
    core.ransac_f8(x1, x2, table, 0.06)
print("ok", core.__file__)
