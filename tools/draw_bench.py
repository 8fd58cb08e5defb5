"""Dev probe (round 4): host MT19937 replay of the RANSAC draw (cfg2: 16384
8-point samples of 5000) -- sfm_pyrandom_sample_table, median of 50 calls.
Runs without a GPU.  Usage: draw_bench.py"""
import os, sys, time, random
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c
random.seed(0)
ts = []
for _ in range(50):
    t = time.perf_counter()
    c.sample_table(5000, 8, 16384)
    ts.append(time.perf_counter() - t)
print(f"sample_table(5000, 8, 16384): median {np.median(ts)*1e3:.4f} ms, min {min(ts)*1e3:.4f} ms "
      f"(SFM_PYRANDOM_CSTORE={os.environ.get('SFM_PYRANDOM_CSTORE', '0')}, "
      f"SFM_PYRANDOM_SCALAR={os.environ.get('SFM_PYRANDOM_SCALAR', '0')})")
