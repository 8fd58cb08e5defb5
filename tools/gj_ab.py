"""Dev probe (round 3): A/B of a BA setting (SFM_* variable) on one box -- the BA
solve at cfg4 / cfg5 (20 fixed LM iterations, HIP-event kernel split),
alternating the environment variable given on the command line between its
values, several rounds.  Usage: gj_ab.py VAR v1,v2 [rounds [pkgdir]]"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, sys.argv[4] if len(sys.argv) > 4 else R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
var, vals = sys.argv[1], sys.argv[2].split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
probs = {}
for name in ("cfg4", "cfg5"):
    p = syn.ba_problem_cfg(name, dense=False)
    probs[name] = (np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])]), p)
res = {}
for r in range(rounds):
    for v in vals:
        os.environ[var] = v
        for name, (cams0, p) in probs.items():
            prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
            prob.solve(max_iterations=3, fixed_iterations=True)
            prob.reset()
            prob.set_timing()
            rep = prob.solve(max_iterations=20, fixed_iterations=True)
            kt = prob.kernel_times()
            prob.close()
            res.setdefault((name, v), []).append(kt)
            print(f"round {r} {var}={v} {name}: " + " ".join(f"{a} {b:.4f}" for a, b in kt.items()) +
                  f" cost {rep['cost']:.10e}", flush=True)
for k, t in sorted(res.items()):
    print(k, "median ms", {a: round(float(np.median([x[a] for x in t])), 4) for a in t[0]})
