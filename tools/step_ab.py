"""Dev probe (round 6): A/B of whole BA bench steps between builds and
environment settings, interleaved on one box.  Each variant runs in a child
process (one _sfmcore per process): bench.py's BA leg -- reset, 3 warmup LM
iterations, then 20 fixed iterations from x0, timed 5 times -- and prints
ms per step (median of the 5) and the fixed-iteration kernel split.
Usage: step_ab.py cfg rounds pkgdir[:VAR=val[,VAR=val]] ..."""
import os, subprocess, sys, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    cfg, pkg = sys.argv[2], sys.argv[3]
    sys.path.insert(0, pkg)
    sys.path.insert(1, R + "/structure-from-motion-_amd")
    import time, numpy as np, _sfmcore as c, sfm_synthetic as syn
    p = syn.ba_problem_cfg(cfg, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
    prob.reset()
    prob.solve(max_iterations=3, fixed_iterations=True)
    ts = []
    for _ in range(5):
        prob.reset()
        t0 = time.perf_counter()
        rep = prob.solve(max_iterations=20, fixed_iterations=True)
        ts.append((time.perf_counter() - t0) * 1e3 / 20)
    prob.reset()
    prob.set_timing(True)
    prob.solve(max_iterations=20, fixed_iterations=True)
    kt = prob.kernel_times()
    prob.close()
    print(json.dumps({"ms": sorted(ts)[2], "all": [round(t, 4) for t in ts], "accepted": rep["accepted"],
                      "cost": rep["cost"], "kt": kt}))
    sys.exit(0)
cfg, rounds, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
res = {}
for r in range(rounds):
    for v in variants:
        pkg, _, envs = v.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, val = kv.partition("=")
            env[k] = val
        out = subprocess.run([sys.executable, __file__, "--child", cfg, os.path.join(R, pkg)], env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stdout, out.stderr)
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res.setdefault(v, []).append(d["ms"])
        print(f"round {r} {cfg} {v}: {d['ms']:.4f} ms/step {d['all']} accepted {d['accepted']} cost {d['cost']:.10e} "
              + " ".join(f"{a} {b:.4f}" for a, b in d["kt"].items()), flush=True)
for v, t in res.items():
    print(cfg, v, "median ms/step", round(sorted(t)[len(t) // 2], 4), "all", [round(x, 4) for x in t])
