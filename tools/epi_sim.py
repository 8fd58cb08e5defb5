"""CPU model of the RANSAC F score's float prefilter at cfg2 (5000 corr,
thr 0.06): per hypothesis (oracle F of the first NH sample rows), the share
of 128-pair passes (and of 256 / 512-pair blocks) in which some pair is not
proven an outlier, for the current test (e^2 > q1 qa + q0) and for the
cheaper one that bounds qa by the block's maximum (|e| > T_block).  Float
arithmetic is modelled in float32 without fma (statistics only)."""
import os
import random
import sys

import numpy as np

_here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_here, "structure-from-motion-_amd"), os.path.join(_here, "oracle")]
import oracle as O  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

NH = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
x1, x2, _, _ = syn.two_view(n=5000, seed=0)
random.seed(0)
rows = np.array([random.sample(range(5000), 8) for _ in range(NH)])
Fs = np.stack([O.f8(x1[r], x2[r]).ravel() for r in rows])
thr_hi2 = 2 * 0.06 * (1 + 1e-4)
b = np.abs(np.concatenate([x1, x2], 1)).max(0)  # X, Y, U, V
X, Y, U, V = [float(np.float32(v)) for v in b]
f32 = np.float32
x, y, u, v = [f32(a) for a in (x1[:, 0], x1[:, 1], x2[:, 0], x2[:, 1])]
n = len(x)
npass = n // 128
stats = {k: [] for k in ("pre128", "pre256", "pre512", "cheap128", "cheap512", "cheap_then_pre512", "inl")}
for f in Fs:
    m = np.abs(f).max()
    ex = np.frexp(m)[1] - 1
    g = np.ldexp(f, -ex - 1)
    c = np.ldexp(1e-8, -ex - 1)
    A0 = abs(g[0]) * X + abs(g[1]) * Y + abs(g[2])
    A1 = abs(g[3]) * X + abs(g[4]) * Y + abs(g[5])
    A2 = abs(g[6]) * X + abs(g[7]) * Y + abs(g[8])
    Mt = U * A0 + V * A1 + A2
    At = np.hypot(A0, A1)
    E = 5e-7 * Mt + 2.0 ** -70
    K1 = thr_hi2 * (1 + 1e-6)
    K0 = thr_hi2 * (3e-7 * At + 2.0 ** -60 + c) + E
    d = 2.0 ** -8
    q1 = f32((1 + d) * K1 * K1 * (1 + 2 ** -20))
    q0 = f32((1 + 1 / d) * K0 * K0 * (1 + 2 ** -20))
    gg = f32(g)
    a0 = gg[1] * y + (gg[0] * x + gg[2])
    a1 = gg[4] * y + (gg[3] * x + gg[5])
    a2 = gg[7] * y + (gg[6] * x + gg[8])
    e = u * a0 + (v * a1 + a2)
    qa = a0 * a0 + a1 * a1
    out = e * e > q1 * qa + q0
    stats["inl"].append(int((~out).sum()))
    o = out[:npass * 128]
    stats["pre128"].append((~o.reshape(-1, 128).all(1)).mean())
    stats["pre256"].append((~o[:npass // 2 * 256].reshape(-1, 256).all(1)).mean())
    stats["pre512"].append((~o[:npass // 4 * 512].reshape(-1, 512).all(1)).mean())
    # cheap: per 512-pair block, qa bounded by the block's float max (a
    # per-block constant would come from the block's coordinate bounds)
    for blk, key in ((128, "cheap128"), (512, "cheap512")):
        nb = len(o) // blk
        qb = qa[:nb * blk].reshape(nb, blk).max(1, keepdims=True)
        T = q1 * qb + q0
        oc = (e[:nb * blk].reshape(nb, blk) ** 2 > T)
        stats[key].append((~oc.all(1)).mean())
        if blk == 512:
            stats["cheap_then_pre512"].append(((~oc) & ~o[:nb * blk].reshape(nb, blk)).any(1).mean())
for k, vals in stats.items():
    a = np.array(vals, dtype=float)
    print(f"{k:18s} mean {a.mean():.4f}  median {np.median(a):.4f}  p90 {np.quantile(a, 0.9):.4f}")
