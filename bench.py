"""Benchmark of the MI355X SfM hot path (BASELINE.json metric:
"BA LM-iterations/sec + RANSAC hypotheses/sec at 1/2/4/8 MI355X; final
reproj RMSE vs ref").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg4|cfg5]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Workload (BASELINE config 4, the one the north-star target is quoted on):
synthetic BA, 50 cameras / 100k points / 1M observations (sfm_synthetic).
A step is one LM iteration (damped Schur solve + trial evaluation, plus the
re-linearisation after an accepted step) of the sparse Schur-complement LM,
with the problem resident in HBM.  N > 1: points are sharded across ranks
(strong scaling of the same problem) with one RCCL all-reduce of the
reduced camera system per iteration.  value = LM iterations / s of the job.

Also reported: RANSAC hypotheses/s on config 2 (5000 correspondences, 40 %
outliers, 16384 hypotheses) on rank 0's GPU; the converged RMSE vs the
reference's least-squares oracle; the roofline of the dominant kernel
(HIP-event time on the library's own stream); a CPU baseline (the C oracle,
1 thread, rank 0 at N = 1).
"""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "structure-from-motion-_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before libsfmcore: one HIP runtime per process)

import _sfmcore as core  # noqa: E402
import sfm_dist  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector


SWEEP_RANGES = 8  # k_schur_sweep's point ranges (SFM_SWEEP_RANGES default)


def algorithmic_bytes(name, n_obs, n_pts, n_pairs, nblocks, ns):
    """Compulsory bytes one launch of each single-kernel family moves
    (DESIGN.md §4): every array the kernel must read or write, once.
    n_pairs: off-diagonal co-observation pairs; nblocks: camera blocks i <= j."""
    if name == "schur_blocks":  # k_schur_sweep + finish: Schur records (p, G, q) 128 B/obs staged once,
        # staged-slot list 4 B/obs, pair list 4 B/pair, range slab written + read, payload written
        return 128 * n_obs + 4 * n_obs + 4 * n_pairs + 2 * 336 * SWEEP_RANGES * nblocks + 8 * (ns * ns + 3 * ns)
    if name == "point_prep":    # J 96 B + cam 4 B read, Schur record 128 B written per obs; V,g / L,q per pt
        return (96 + 4 + 128) * n_obs + (72 + 72 + 4) * n_pts
    if name == "linearize":     # k_linearize: obs, cam read, J 96 B written per obs; X, V,g per pt
        # + k_camera_lin: J 96 B + camera-major index 4 B per obs
        return (16 + 4 + 96) * n_obs + (24 + 72 + 4) * n_pts + (96 + 4) * n_obs
    if name == "backsub_trial": # J, obs, cam per obs; V,g, L,q, X, X' per pt
        return (96 + 16 + 4) * n_obs + (72 + 72 + 24 + 24 + 4) * n_pts
    return None


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (tools/profile_round.sh + tools/pmc_summary.py), or None."""
    names = {"schur_blocks": "k_schur_sweep", "point_prep": "k_point_prep", "linearize": "k_linearize",
             "backsub_trial": "k_backsub_trial"}
    path = os.path.join(REPO, "profiles", "round1", "pmc_traffic.json")
    try:
        d = json.load(open(path)).get(names.get(kernel, kernel), {})
        v = d.get("hbm_bytes_per_launch")
        return int(v) if v else None
    except (OSError, ValueError):
        return None


def n_pairs_of(pt_idx):
    """off-diagonal co-observation pairs (two observations of one point)"""
    k = np.bincount(pt_idx)
    return int((k * (k - 1) // 2).sum())


def cpu_baseline_ba(prob, K):
    import oracle as O  # test infrastructure: the CPU restatement, timed as the baseline
    cams0 = np.column_stack([prob["rotvec0"], np.einsum("nij,nj->ni", -prob["R0"], prob["C0"])])
    t = time.perf_counter()
    _, _, rep = O.ba_lm(cams0, prob["X0"], prob["cam_idx"], prob["pt_idx"], prob["obs"], K, max_iterations=50)
    dt = time.perf_counter() - t
    return rep["iterations"] / dt, rep, dt


def cpu_baseline_ransac(x1, x2, samples):
    import oracle as O
    t = time.perf_counter()
    O.ransac(x1, x2, samples, 0.06)
    dt = time.perf_counter() - t
    return len(samples) / dt, dt


K = syn.K_REF


def next_rows(core, local_rank, cpu):
    """§8(f) rows, rank 0: GPU throughput of each (kernel-only and end to
    end through the C-ABI), and -- in the cpu_baseline leg only -- the C
    oracle on a bounded sample of the same workload."""
    if cpu:
        import oracle as O  # test infrastructure: the CPU restatement, timed as the baseline
    out = {}
    x1, x2, _, m = syn.two_view(n=1_000_000, seed=6, outlier_frac=0.2)
    P1 = K @ np.hstack([np.eye(3), np.zeros((3, 1))])
    P2 = K @ np.hstack([m["R2"], (-m["R2"] @ m["C2"]).reshape(3, 1)])
    X0 = core.triangulate(P1, P2, x1, x2)
    core.triangulate_nonlinear(P1, P2, x1[:1000], x2[:1000], X0[:1000])
    t = time.perf_counter()
    core.triangulate_nonlinear(P1, P2, x1, x2, X0)
    te = time.perf_counter() - t
    tk = core.last_timings()[1] * 1e-3
    r = {"workload": "1M two-view points, 20% outliers, DLT start, max_nfev=50",
         "points_per_s_kernel": round(len(x1) / tk, 1), "points_per_s_end_to_end": round(len(x1) / te, 1)}
    if cpu:
        t = time.perf_counter()
        O.nltri(K, np.zeros(3), np.eye(3), m["C2"], m["R2"], x1[:200_000], x2[:200_000], X0[:200_000])
        r["cpu_oracle_points_per_s"] = round(200_000 / (time.perf_counter() - t), 1)
        r["cpu_sample"] = "C oracle lmdif (oracle/sfm_oracle_lm.c), 200k points, 1 thread"
    out["nonlinear_triangulation"] = r
    # homography RANSAC, cfg2 correspondences, 16384 hypotheses, thr 30
    h1, h2, _, _ = syn.two_view(n=5000, seed=0)
    random.seed(0)
    hs = core.sample_table(5000, 4, 16384)
    core.ransac_h4(h1, h2, hs, 30.0)
    core.ransac_h4(h1, h2, hs, 30.0)
    tk = core.last_timings()[1] * 1e-3
    random.seed(0)
    core.ransac_h4_pyrandom(h1, h2, 16384, 30.0)  # the drop-in's call: in-call sampling
    random.seed(0)
    t = time.perf_counter()
    core.ransac_h4_pyrandom(h1, h2, 16384, 30.0)
    te = time.perf_counter() - t
    r = {"workload": "cfg2 5000 corr, 16384 4-point hypotheses, thr 30",
         "hyps_per_s_kernels": round(16384 / tk, 1), "hyps_per_s_end_to_end": round(16384 / te, 1)}
    if cpu:
        t = time.perf_counter()
        O.ransac_h(h1, h2, hs[:1024], 30.0)
        r["cpu_oracle_hyps_per_s"] = round(1024 / (time.perf_counter() - t), 1)
    out["homography_ransac"] = r
    # PnP RANSAC + NonlinearPnP on 5000 world points (30 % outliers)
    rng = np.random.default_rng(12)
    n = 5000
    Xw = np.column_stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)])
    u = (K @ (m["R2"] @ (Xw - m["C2"]).T)).T
    xw = u[:, :2] / u[:, 2:3] + rng.normal(0, 0.5, (n, 2))
    o = rng.choice(n, n * 3 // 10, replace=False)
    xw[o] = rng.uniform(0, 1000, (len(o), 2))
    random.seed(1)
    ps = core.sample_table(n, 4, 16384)
    core.pnp_ransac(Xw, xw, K, ps, 8.0)
    t = time.perf_counter()
    _, _, C, R, _, _ = core.pnp_ransac(Xw, xw, K, ps, 8.0)
    te = time.perf_counter() - t
    tk = core.last_timings()[1] * 1e-3
    t = time.perf_counter()
    core.nonlinear_pnp(Xw, xw, K, C, R)
    tn = time.perf_counter() - t
    r = {"workload": "5000 points, 30% outliers, 16384 4-point hypotheses, thr 8; NonlinearPnP max_nfev=100",
         "hyps_per_s_kernels": round(16384 / tk, 1), "hyps_per_s_end_to_end": round(16384 / te, 1),
         "nonlinear_pnp_ms": round(tn * 1e3, 3)}
    if cpu:
        t = time.perf_counter()
        O.pnp_ransac(Xw, xw, K, ps[:1024], 8.0)
        r["cpu_oracle_hyps_per_s"] = round(1024 / (time.perf_counter() - t), 1)
        t = time.perf_counter()
        O.nonlinear_pnp(Xw, xw, K, C, R)
        r["cpu_oracle_nonlinear_pnp_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    out["pnp"] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg4", choices=["cfg3", "cfg4", "cfg5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ransac-hyps", type=int, default=16384)
    ap.add_argument("--force-comm", action="store_true", help="use the RCCL communicator even with one rank")
    ap.add_argument("--no-next-rows", action="store_true", help="skip the SURVEY §8(f) row measurements")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    assert torch.cuda.is_available(), "bench.py needs an MI355X"
    torch.cuda.set_device(local_rank)
    core.require_device()

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    def allmax(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t.item())

    # ---------------- BA workload (every rank generates the same problem)
    K = syn.K_REF
    prob = syn.ba_problem_cfg(args.workload, dense=False)
    cams0 = np.column_stack([prob["rotvec0"], np.einsum("nij,nj->ni", -prob["R0"], prob["C0"])])
    ci, pi, ob, X0, (lo, hi) = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"],
                                                 world, rank)
    comm = None
    if world > 1 or args.force_comm:
        uid = [core.Comm.unique_id() if rank == 0 else None]
        if world > 1:
            torch.distributed.broadcast_object_list(uid, src=0)
        comm = core.Comm(uid[0], world, rank, device=local_rank)
    ba = core.BAProblem(cams0, X0, ci, pi, ob, K, comm=comm, device=local_rank)

    # converged solve (RMSE vs the reference's least-squares solution)
    conv = ba.solve(max_iterations=100)
    n_obs_total = len(prob["cam_idx"])
    rmse0 = syn.rmse_from_cost(conv["cost0"], n_obs_total)
    rmse = syn.rmse_from_cost(conv["cost"], n_obs_total)

    # warmup, then exactly K timed LM iterations from the initial state
    ba.reset()
    ba.solve(max_iterations=args.warmup, fixed_iterations=True)
    ba.reset()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rep = ba.solve(max_iterations=args.steps, fixed_iterations=True)
    torch.cuda.synchronize()
    barrier()
    dt = allmax(time.perf_counter() - t0)
    ktimes = ba.kernel_times()
    ba.close()
    if comm is not None:
        comm.close()

    # ---------------- RANSAC (config 2) on this rank's GPU
    x1, x2, idx, _ = syn.two_view(n=5000, seed=0)
    random.seed(0)
    samples = core.sample_table(5000, 8, args.ransac_hyps)
    for _ in range(3):
        core.ransac_f8(x1, x2, samples, 0.06, device=local_rank)
    reps = 20
    # end to end = the drop-in's whole call: the samples drawn from the global
    # random stream inside it (chunked, overlapped with the GPU), upload,
    # kernels, mask download
    for _ in range(3):
        random.seed(0)
        core.ransac_f8_pyrandom(x1, x2, args.ransac_hyps, 0.06, device=local_rank)
    t = time.perf_counter()
    for _ in range(reps):
        random.seed(0)
        best, F, mask, _, _ = core.ransac_f8_pyrandom(x1, x2, args.ransac_hyps, 0.06, device=local_rank)
    t_e2e = (time.perf_counter() - t) / reps
    t_draw = core.last_timings()[6]
    kt = []
    for _ in range(reps):
        core.ransac_f8(x1, x2, samples, 0.06, device=local_rank)
        tm = core.last_timings()
        kt.append((tm[1], tm[3]))
    k_all, k_score = np.median([a for a, _ in kt]), np.median([b for _, b in kt])

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    n_pairs = n_pairs_of(prob["pt_idx"][prob["pt_idx"] < hi] if world > 1 else prob["pt_idx"])
    ns = 6 * prob["n_cams"]
    nblocks = prob["n_cams"] * (prob["n_cams"] + 1) // 2
    # dominant single kernel (the Cholesky family is a chain of ~2 launches
    # per 16-column panel, latency-bound; it is reported in kernel_ms_per_iter)
    fam = {k: v for k, v in ktimes.items() if algorithmic_bytes(k, 1, 1, 1, 1, 1) is not None}
    dom = max(fam, key=fam.get)
    n_obs_local, n_pts_local = len(ci), len(X0)
    alg = algorithmic_bytes(dom, n_obs_local, n_pts_local, n_pairs, nblocks, ns)
    ach = alg / (ktimes[dom] * 1e-3) / 1e9
    # the committed PMC pass is of the default single-GPU cfg4 run; other
    # workloads / shardings have other per-launch traffic
    traffic = pmc_traffic(dom) if (args.workload == "cfg4" and world == 1) else None
    roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "algorithmic_bytes": int(alg),
            "avg_launch_ms": round(ktimes[dom], 4),
            "traffic_source": "profiles/round1/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE, "
                              "(2*FETCH+WRITE) KiB per launch)"}
    iter_bytes = 52 * n_obs_total + 240 * prob["n_pts"]  # SURVEY §8(d) compulsory bytes / LM iteration
    ms_per_step = dt / args.steps * 1e3
    out = {
        "metric": "BA LM-iterations/sec (+ RANSAC hypotheses/sec, final reproj RMSE vs ref)",
        "value": round(args.steps / dt, 3),
        "unit": "LM-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (sfm_synthetic.ba_problem, seed 3)",
        "config": {"workload": f"{args.workload}: BA {prob['n_cams']} cams / {prob['n_pts']} pts / "
                               f"{n_obs_total} obs, Schur-complement LM, points sharded over {world} rank(s)",
                   "parallelism": f"point-shard x{world} + RCCL all-reduce of the reduced camera system"},
        "roofline": roof,
        "kernel_ms_per_iter": {k: round(v, 4) for k, v in ktimes.items()},
        "iteration_roofline": {"compulsory_bytes": iter_bytes,
                               "achieved_GBs": round(iter_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                               "frac": round(iter_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
        "rmse": {"initial": round(rmse0, 6), "converged": round(rmse, 6), "lm_iterations": conv["iterations"],
                 "note": "cfg3 parity vs the reference least-squares oracle in tests/test_gpu_parity.py"},
        "ransac": {"workload": "cfg2: 5000 corr, 40% outliers", "hypotheses": args.ransac_hyps,
                   "hyps_per_s_end_to_end": round(args.ransac_hyps / t_e2e, 1),
                   "host_sampling_ms": round(float(t_draw), 3),
                   "hyps_per_s_kernels": round(args.ransac_hyps / (k_all * 1e-3), 1),
                   "score_kernel_ms": round(float(k_score), 4), "best_iter": int(best), "inliers": int(mask.sum())},
    }
    cpu_leg = world == 1 and not args.no_cpu_baseline
    if cpu_leg:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
    if not args.no_next_rows:
        out["next_rows"] = next_rows(core, local_rank, cpu_leg)
    if cpu_leg:
        v, crep, cdt = cpu_baseline_ba(prob, K)
        hs = samples[:1024]
        rv, rdt = cpu_baseline_ransac(x1, x2, hs)
        out["cpu_baseline"] = {"value": round(v, 4), "unit": "LM-iterations/s", "cores": 1, "kind": "port",
                               "sample": f"C oracle Schur-LM (oracle/sfm_oracle.c), full {args.workload} problem, "
                                         f"{crep['iterations']} LM iterations to convergence in {cdt:.1f}s, 1 thread",
                               "speedup": round(out["value"] / v, 1),
                               "ransac_hyps_per_s": round(rv, 1),
                               "ransac_sample": f"C oracle, 1024 cfg2 hypotheses in {rdt:.2f}s, 1 thread",
                               "cpu": _cpu_model(), "os_cpu_count": os.cpu_count()}
    print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
