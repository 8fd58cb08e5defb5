"""Dev probe (round 6): the BA drop-in's whole call (bench.end_to_end_ba) with
two builds of the library on one box, alternated over rounds, each run in a
child process (one libsfmcore per process).  The build is the package
directory whose _sfmcore / libsfmcore.so the child imports first.
A build may carry environment settings: pkgdir:VAR=value[,VAR=value].
Usage: e2e_ab.py cfg5 rounds pkgdir_a pkgdir_b"""
import json
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    cfg, pkg = sys.argv[2], sys.argv[3]
    sys.path.insert(0, pkg)
    import _sfmcore  # noqa: F401  (this build and its drop-in, before bench puts its own package first)
    import BundleAdjustment  # noqa: F401
    sys.path.insert(0, R)
    import bench
    print(json.dumps(bench.end_to_end_ba(cfg)), flush=True)
    sys.exit(0)
cfg, rounds, pkgs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
res = {p: [] for p in pkgs}
for r in range(rounds):
    for p in pkgs:
        d, _, kv = p.partition(":")
        env = dict(os.environ, SFM_CREATE_TIMING="1", **dict(a.split("=", 1) for a in kv.split(",") if a))
        out = subprocess.run([sys.executable, "-u", __file__, "--child", cfg, d], capture_output=True, text=True,
                             timeout=600, env=env)
        if out.returncode != 0:
            print(out.stderr[-2000:], flush=True)
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        ph = d["phases_ms"]
        res[p].append(d["total_ms"])
        create = [l for l in out.stderr.splitlines() if l.startswith("[create]")]
        print(f"round {r} {p}: total {d['total_ms']:.2f} ms  obs {ph.get('observations', 0):.2f}  create "
              f"{ph.get('ba_lm_create', 0):.2f}  loop {ph.get('ba_lm_loop', 0):.2f}", flush=True)
        for l in create[-15:]:
            print("    " + l, flush=True)
for p, v in res.items():
    print(f"{p}: totals {['%.2f' % x for x in v]} min {min(v):.2f}", flush=True)
