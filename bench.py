"""Benchmark of the MI355X SfM hot path (BASELINE.json metric:
"BA LM-iterations/sec + RANSAC hypotheses/sec at 1/2/4/8 MI355X; final
reproj RMSE vs ref").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg5|cfg4|cfg3]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Headline workload (value): BASELINE config 5, the config the 1/2/4/8 scaling
curve is quoted on -- synthetic BA, 200 cameras / 500k points / 4M
observations (sfm_synthetic) -- at every N, so the driver's per-N values
form that curve.  A step is one LM iteration (damped Schur solve + trial
evaluation, plus the re-linearisation after an accepted step) of the sparse
Schur-complement LM with the problem resident in HBM.  N > 1: points are
sharded across ranks (strong scaling of the same problem), one RCCL
all-reduce of the reduced camera system per iteration.  value = LM
iterations / s of the job.

Also reported: the same record for BASELINE config 4 (50 cams / 100k pts /
1M obs, the config of the north-star >= 50x target) under "cfg4"; RANSAC
hypotheses/s on config 2 (5000 correspondences, 40 % outliers, 16384
hypotheses); converged RMSE vs the reference's least-squares oracle; the
roofline of the LM iteration; the CPU baselines of SURVEY §8(d) (rank 0,
N = 1): the OpenMP Schur-LM and RANSAC on the host's threads (a thread
sweep), the 1-thread C oracle, the reference's own loop extrapolated.
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


def sweep_ranges(ns, ncu=256):
    """k_schur_sweep's point ranges as plan_sweep picks them (csrc/ba.hip): the
    largest of 8, 4, 2, 1 with specs x ranges <= the CU count, a spec being
    two camera rows (nc / 2 rounded up) -- 8 at cfg4, 2 at cfg5."""
    nc = ns // 6
    nspec = (nc + 1) // 2
    for nr in (8, 4, 2, 1):
        if nspec * nr <= ncu:
            return nr
    return 8


def design_bytes(name, n_obs, n_pts, n_pairs, nblocks, ns):
    """Bytes one launch of each kernel family must move in THIS design
    (DESIGN.md §4's table: no stored Jacobians, no per-observation records
    -- the record-free sweep), per LM iteration -- reported next to the SURVEY
    §8(d) compulsory bytes, which are the roofline's.  n_pairs: off-diagonal
    co-observation pairs; nblocks: camera blocks i <= j."""
    if name == "schur_blocks":  # k_schur_sweep: X (24 B) + Lq (72 B) gathered per staged observation, the
        # obs index read (4 B/obs), pair list 2 B/pair, range slab written + read, payload written
        return 100 * n_obs + 2 * n_pairs + 2 * 336 * sweep_ranges(ns) * nblocks + 8 * (ns * ns + 3 * ns)
    if name == "point_prep":    # V, g read, L, q (Lq) written per point
        return 144 * n_pts
    if name == "linearize":     # k_linearize: obs + cam (24 B/obs incl. the point CSR), X in, V, g out per point;
        # camera blocks (in the sweep launch): camera-major pt + obs (20 B) + X gather (24 B) per obs
        return 24 * n_obs + 100 * n_pts + 44 * n_obs
    if name == "backsub_trial": # cam + obs per obs (the Jacobians recomputed); V,g, L,q, X, X' per pt
        return 20 * n_obs + 196 * n_pts
    if name == "cholesky":      # the persistent Gauss-Jordan solve: the damped system read once, every
        # panel (G rows of all nsp rows x 16) written once and read by the column blocks it updates
        nt = (ns + 15) // 16
        return 8 * (ns * ns // 2 + 2 * nt * nt * 16 * 16)
    return None


PMC_ROUND = "round6"

# VALU issue (MI355X_MICROARCH.md): a SIMD issues a wave64 VALU instruction
# over 2 cycles (32 lanes a cycle); an FP64 op takes the slot twice (78.6 TF
# FP64 vector = 16 lanes a cycle), a transcendental four times
VALU_SLOTS_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 issue slots / s, the whole chip


def ransac_valu_slots():
    """Executed VALU issue slots of the F-RANSAC kernels from the committed
    rocprofv3 PMC passes (SQ_INSTS_VALU and the FP64 / transcendental splits):
    the one-shot score launch (16,384 x 5,000) and the drop-in call's own fits
    + scores (tools/ransac_once.py), per launch / per call.
    ({"oneshot": slots, "dropin": slots}, sources)."""
    import csv
    out, src = {}, []
    base = os.path.join(REPO, "profiles", PMC_ROUND)
    try:
        per = {}
        for r in csv.DictReader(open(os.path.join(base, "ransac_oneshot_pmc", "pmc_counter_collection.csv"))):
            if "k_epi_score" in r["Kernel_Name"]:
                per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        if per.get("SQ_INSTS_VALU"):  # FP64 ops take 2 slots, FP64 transcendentals 4 (the pass has the splits
            # since round 6; round 5's had SQ_INSTS_VALU alone, one slot each)
            m = {k: float(np.mean(v)) for k, v in per.items()}
            out["oneshot"] = (m["SQ_INSTS_VALU"] + sum(m.get(f"SQ_INSTS_VALU_{c}_F64", 0.0) for c in ("ADD", "FMA", "MUL"))
                              + 3 * m.get("SQ_INSTS_VALU_TRANS_F64", 0.0))
            src.append(f"profiles/{PMC_ROUND}/ransac_oneshot_pmc (k_epi_score: SQ_INSTS_VALU + the FP64 splits, "
                       f"tools/ransac_oneshot.py)")
    except (OSError, ValueError, KeyError):
        pass
    try:
        d = json.load(open(os.path.join(base, "pmc_traffic_ransac.json")))
        calls = d["void k_fit_samples<EpiModel>"]["launches"]  # one first-chunk fit per drop-in call
        tot = 0.0
        for k in ("void k_epi_score<true>", "void k_epi_score<false>", "void k_fit_samples<EpiModel>"):
            e = d[k]
            f64 = sum(e.get(f"SQ_INSTS_VALU_{c}_F64_total", 0.0) for c in ("ADD", "FMA", "MUL"))
            tot += e["SQ_INSTS_VALU_total"] + f64 + 3 * e.get("SQ_INSTS_VALU_TRANS_F64_total", 0.0)
        out["dropin"] = tot / calls
        src.append(f"profiles/{PMC_ROUND}/pmc_traffic_ransac.json (the drop-in's fits + scores per call; FP64 "
                   f"ops 2 slots, FP64 transcendentals 4)")
    except (OSError, ValueError, KeyError):
        pass
    return out, src


def pmc_iteration(workload):
    """HBM bytes per LM iteration by kernel from the committed rocprofv3 PMC
    passes of tools/ba_once.py (the workload, 20 fixed iterations from x0 --
    the timed region's mix): ({kernel: bytes per iteration}, source path), or
    ({}, None)."""
    for rnd, name in ((PMC_ROUND, f"pmc_iteration_{workload}.json"),
                      ("round2", "pmc_iteration.json" if workload == "cfg4" else None)):
        if name is None:
            continue
        path = os.path.join(REPO, "profiles", rnd, name)
        try:
            return json.load(open(path)).get("bytes_per_iteration", {}), f"profiles/{rnd}/{name}"
        except (OSError, ValueError):
            continue
    return {}, None


def n_pairs_of(pt_idx):
    """off-diagonal co-observation pairs (two observations of one point)"""
    k = np.bincount(pt_idx)
    return int((k * (k - 1) // 2).sum())


def ba_flops(pt_idx, n_cams):
    """SURVEY §8(d) FP64 work of one LM iteration: 400 N_obs (linearise,
    eliminate, back-substitute, trial cost) + sum_p (108 k_p + 216 k_p (k_p+1)/2)
    (per-point W V^-1 W^T blocks) + (6 n_c)^3 / 3 (the reduced solve)."""
    k = np.bincount(pt_idx).astype(np.float64)
    return float(400 * len(pt_idx) + (108 * k + 216 * k * (k + 1) / 2).sum() + (6 * n_cams) ** 3 / 3)


def _physical_cores():
    """Physical cores behind the CPUs this process may use (sysfs core ids),
    or None where sysfs does not say."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
        ids = set()
        for c in cpus:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            ids.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        return {"physical": len(ids), "logical": len(cpus)}
    except OSError:
        return None


def cpu_baseline_ba(prob, cams0, sweep, single=True):
    """The CPU legs of SURVEY §8(d) for the BA (rank 0, N = 1; test
    infrastructure only -- the oracle is the checker and the baseline, never
    the product):
      * CPU-strong: the OpenMP Schur-LM (oracle/sfm_cpu_strong.c) at every
        thread count of `sweep`; at cfg4 to convergence, at cfg5 a bounded 3
        iterations per point (LM-it/s = iterations / wall time; the 1-thread
        point alone would take minutes to converge), then the sweep's fastest
        thread count again to convergence;
      * (single) the 1-thread C Schur-LM (oracle/sfm_oracle.c) to convergence;
      * the reference's own path priced by its residual loop
        (oracle/ref_loop.py, the reference loop structure call for call) on a
        bounded sample of observations: one lmdif Jacobian = (n + 1)
        residual evaluations (extrapolated, labelled as such)."""
    import oracle as O  # test infrastructure: the CPU restatement, timed as the baseline
    import ref_loop
    args = (cams0, prob["X0"], prob["cam_idx"], prob["pt_idx"], prob["obs"], K)
    iters = 50 if single else 3
    strong = {}
    for t in sweep:
        O.set_threads(t)
        t0 = time.perf_counter()
        _, _, srep = O.ba_lm_cpu_strong(*args, max_iterations=iters)
        ts = time.perf_counter() - t0
        strong[t] = (srep["iterations"] / ts, srep, ts)
    out = dict(strong=strong)
    if not single:  # cfg5: the fastest thread count to convergence
        best_t = max(strong, key=lambda t: strong[t][0])
        O.set_threads(best_t)
        t0 = time.perf_counter()
        _, _, crep = O.ba_lm_cpu_strong(*args, max_iterations=50)
        ts = time.perf_counter() - t0
        out["converged"] = (crep["iterations"] / ts, crep, ts, best_t)
    O.set_threads(max(sweep))
    if single:
        t0 = time.perf_counter()
        _, _, orep = O.ba_lm(*args, max_iterations=50)
        to = time.perf_counter() - t0
        out["oracle"] = (orep["iterations"] / to, orep, to)
    # reference residual loop on a bounded sample of observations
    n_s = 20000
    nc, npt = prob["n_cams"], prob["n_pts"]
    params = np.concatenate([cams0.ravel(), prob["X0"].ravel()])
    t0 = time.perf_counter()
    ref_loop.residuals(params, nc, npt, prob["cam_idx"][:n_s], prob["pt_idx"][:n_s], prob["obs"][:n_s], K)
    per_obs = (time.perf_counter() - t0) / n_s
    n_par = 6 * nc + 3 * npt
    eval_s = per_obs * len(prob["cam_idx"])
    out["ref"] = dict(per_obs_us=per_obs * 1e6, eval_s=eval_s, n_params=n_par,
                      jacobian_s=eval_s * (n_par + 1), sample_obs=n_s)
    return out


def cpu_cfg3_as_shipped():
    """The reference as shipped at cfg3 (6 cams / 2000 pts / 10k obs):
    MINPACK lmdif with max_nfev=100 = (3n + 2) residual evaluations (n + 1
    for the Jacobian, 1 trial, 2n for scipy's post-hoc approx_derivative,
    SURVEY §3.3) + a dense QR of the m x n Jacobian.  Composed from the
    timed residual loop and a timed numpy QR of a (m/4) x (n/4) matrix
    scaled by m n^2 (LAPACK's blocked dgeqrf: a lower bound for lmdif's
    unblocked qrfac).  Measured whole in the build container: 3093 s."""
    import ref_loop
    p = syn.ba_problem(6, 2000, 5, seed=3, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    params = np.concatenate([cams0.ravel(), p["X0"].ravel()])
    t = time.perf_counter()
    ref_loop.residuals(params, 6, 2000, p["cam_idx"], p["pt_idx"], p["obs"], K)
    ev = time.perf_counter() - t
    n, m = len(params), 2 * len(p["cam_idx"])
    A = np.random.default_rng(0).standard_normal((m // 4, n // 4))
    t = time.perf_counter()
    np.linalg.qr(A, mode="r")
    qr = (time.perf_counter() - t) * 64
    return {"residual_eval_s": round(ev, 4), "evaluations": 3 * n + 2, "dense_qr_s": round(qr, 2),
            "composed_s": round(ev * (3 * n + 2) + qr, 1), "measured_in_build_container_s": 3092.8,
            "note": "composed = residual_eval x (3n+2) + dense QR (scaled from m/4 x n/4); the reference "
                    "returns x0 unchanged here (SURVEY §0.4)"}


def cpu_baseline_ransac(x1, x2, samples, sweep, thr=0.06):
    """The OpenMP RANSAC (cs_ransac) over the thread sweep, all hypotheses;
    returns the fastest point (hyps/s, seconds, threads)."""
    import oracle as O
    best = None
    for t in sweep:
        O.set_threads(t)
        t0 = time.perf_counter()
        O.ransac_cpu_strong(x1, x2, samples, thr)
        dt = time.perf_counter() - t0
        if best is None or dt < best[1]:
            best = (len(samples) / dt, dt, t)
    O.set_threads(max(sweep))
    return best


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
    # kernel times from a call with HIP events on (sfm_set_call_timing),
    # end-to-end from a call without them
    core.set_call_timing(True)
    core.triangulate_nonlinear(P1, P2, x1, x2, X0)
    tk = core.last_timings()[1] * 1e-3
    core.set_call_timing(False)
    t = time.perf_counter()
    core.triangulate_nonlinear(P1, P2, x1, x2, X0)
    te = time.perf_counter() - t
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
    core.set_call_timing(True)
    core.pnp_ransac(Xw, xw, K, ps, 8.0)
    tk = core.last_timings()[1] * 1e-3
    core.set_call_timing(False)
    t = time.perf_counter()
    _, _, C, R, _, _ = core.pnp_ransac(Xw, xw, K, ps, 8.0)
    te = time.perf_counter() - t
    core.nonlinear_pnp(Xw, xw, K, C, R)  # warm
    tl = []
    for _ in range(5):
        t = time.perf_counter()
        core.nonlinear_pnp(Xw, xw, K, C, R)
        tl.append(time.perf_counter() - t)
    tn = float(np.median(tl))
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


def end_to_end_ba(workload):
    """The drop-in itself, perform_bundle_adjustment (Phase 1/BundleAdjustment.py:113-242),
    on the reference's dense interface: feature_x / feature_y / flag matrices
    (n_pts x n_cams) and R / C lists in, optimised R / C lists and points out,
    run to convergence.  The call is timed whole (host buffers in and out:
    PCIe and host prep included) and split into its phases
    (BundleAdjustment.last_timings).  Second of two calls (the first warms the
    library's thread context)."""
    import contextlib
    import io
    import BundleAdjustment as BA
    p = syn.ba_problem_cfg(workload, dense=False)
    n_pts, n_cams = p["n_pts"], p["n_cams"]
    fx = np.zeros((n_pts, n_cams))
    fy = np.zeros((n_pts, n_cams))
    fl = np.zeros((n_pts, n_cams), dtype=np.int64)
    fx[p["pt_idx"], p["cam_idx"]] = p["obs"][:, 0]
    fy[p["pt_idx"], p["cam_idx"]] = p["obs"][:, 1]
    fl[p["pt_idx"], p["cam_idx"]] = 1
    fwc = np.ones((n_pts, 1), dtype=np.int64)
    R_set, C_set = list(p["R0"]), list(p["C0"])
    runs = []
    for _ in range(1 + E2E_TIMED):
        with contextlib.redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            BA.perform_bundle_adjustment(p["X0"], fwc, fx, fy, fl, R_set, C_set, K, 0)
            dt = time.perf_counter() - t0
        runs.append((dt, dict(BA.last_timings)))
    del fx, fy, fl
    timed = sorted(runs[1:], key=lambda r: r[0])  # the first call warms the library's thread context
    dt, tm = timed[0]
    its = int(tm.get("iterations", 0))
    phases = {k: round(v, 3) for k, v in tm.items() if k not in ("iterations", "total")}
    lib = tm.get("ba_lm", 0.0)
    phases["ba_lm_wrapper"] = round(lib - tm.get("ba_lm_create", 0) - tm.get("ba_lm_loop", 0)
                                    - tm.get("ba_lm_download", 0), 3)
    total = dt * 1e3
    return {"workload": f"{workload}: perform_bundle_adjustment, dense {n_pts} x {n_cams} feature/flag matrices, "
                        f"to convergence",
            "total_ms": round(total, 3), "LM_iterations": its,
            "calls_ms": [round(r[0] * 1e3, 3) for r in runs[1:]],
            "median_ms": round(timed[len(timed) // 2][0] * 1e3, 3),
            "observations_ms_per_call": [round(r[1].get("observations", 0.0), 3) for r in runs[1:]],
            "LM_it_per_s_end_to_end": round(its / dt, 2) if its else None,
            "LM_it_per_s_loop_only": round(its / (tm["ba_lm_loop"] * 1e-3), 2) if its and tm.get("ba_lm_loop") else None,
            "phases_ms": phases,
            "phase_frac": {k: round(v / total, 4) for k, v in phases.items() if not k.startswith("ba_lm_")
                           or k == "ba_lm_create"},
            "note": f"the fastest of {E2E_TIMED} calls after a warm-up call (all listed in calls_ms; the host "
                    "phases, the dense scan above all, vary with the shared host's load, observations_ms_per_call); "
                    "phases: observations = the valid rows and the dense flags -> COO scan (native, host threads), "
                    "cams0 = R -> rotvec and t for the cameras (stacked), pts0 = the valid rows of all_world_coords "
                    "(native gather), ba_lm = the C-ABI call (create: host prep + sweep plan + uploads; loop, whose "
                    "first linearisation is also scipy's non-finite-x0 check; download), post = rotvec -> R, C"}


E2E_TIMED = 3  # timed drop-in calls of end_to_end_ba


def shard_local(workload, steps, warmup):
    """Rank 0's point shard of the workload for N = 2, 4, 8 ranks, run alone
    on this one GPU through a one-rank RCCL communicator (the multi-rank code
    path: the Schur finish launch and the all-reduce call are in, the
    replicated reduced solve too), W warmup + K fixed LM iterations from x0,
    then the per-kernel split with HIP events on.  Bounds the N-GPU step from
    below (no xGMI traffic); the all-reduce over xGMI is given as an estimate
    beside it, labelled so.  The shard's own LM sees a different cost than the
    full problem, so its accept/reject mix is reported too."""
    prob = syn.ba_problem_cfg(workload, dense=False)
    cams0 = np.column_stack([prob["rotvec0"], np.einsum("nij,nj->ni", -prob["R0"], prob["C0"])])
    comm = core.Comm(core.Comm.unique_id(), 1, 0, device=0)
    nc = prob["n_cams"]
    ns = 6 * nc
    payload_bytes = 8 * (36 * nc * (nc + 1) // 2 + 3 * ns)
    out = {"workload": workload, "payload_bytes": payload_bytes}
    try:
        for n in (1, 2, 4, 8):
            ci, pi, ob, X0, (lo, hi) = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"],
                                                         prob["X0"], n, 0)
            ba = core.BAProblem(cams0, X0, ci, pi, ob, K, comm=comm)
            ba.solve(max_iterations=warmup, fixed_iterations=True)
            ba.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rep = ba.solve(max_iterations=steps, fixed_iterations=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ba.reset()
            ba.set_timing(True)
            ba.solve(max_iterations=steps, fixed_iterations=True)
            kt = ba.kernel_times()
            ba.close()
            # ring all-reduce estimate over xGMI (NOT measured): 2 (N-1)/N of the
            # payload at an assumed 300 GB/s bus bandwidth + 15 us latency
            est = (15e-3 + 2 * (n - 1) / n * payload_bytes / 300e9 * 1e3) if n > 1 else 0.0
            ms = dt / steps * 1e3
            out[str(n)] = {"ms_per_step": round(ms, 4), "accepted": rep["accepted"], "n_pts_local": len(X0),
                           "n_obs_local": len(ci), "kernels_ms": {k: round(v, 4) for k, v in kt.items()},
                           "allreduce_ms_estimate": round(est, 4),
                           "ms_per_step_bound": round(ms + est, 4),
                           "LM_it_per_s_bound": round(1e3 / (ms + est), 2)}
    finally:
        comm.close()
    out["note"] = ("rank-0 shard alone on one GPU (1-rank RCCL communicator); ms_per_step_bound = measured + "
                   "all-reduce ESTIMATE (2(N-1)/N x payload / 300 GB/s + 15 us, not measured)")
    return out


def ransac_leg(args, world, rank, local_rank, comm):
    """RANSAC on config 2 (5000 correspondences, 40 % outliers, H = 16384).
    Without a communicator: the drop-in's whole call (in-call sampling from
    the global random stream, upload, kernels, mask download).  With one
    (N > 1, or --force-comm): hypothesis-sharded
    (SURVEY §8(e)): every rank draws the whole table, fits and scores its
    contiguous range, the keys are combined over RCCL and the winner's F
    gives the mask; value = H / (max over ranks of the sharded call)."""
    import sfm_dist
    x1, x2, idx, _ = syn.two_view(n=5000, seed=0)
    H = args.ransac_hyps
    random.seed(0)
    samples = core.sample_table(5000, 8, H)
    reps = 20
    out = {"workload": "cfg2: 5000 corr, 40% outliers", "hypotheses": H}
    if comm is None:
        for _ in range(3):
            core.ransac_f8(x1, x2, samples, 0.06, device=local_rank)
        from GetInliersRANSAC import GetInliersRANSAC  # the drop-in (Phase 1/GetInliersRANSAC.py:5-106)
        for _ in range(3):
            random.seed(0)
            GetInliersRANSAC(x1, x2, idx, 0.06, H)
        t = time.perf_counter()
        for _ in range(reps):
            random.seed(0)
            GetInliersRANSAC(x1, x2, idx, 0.06, H)
        t_e2e = (time.perf_counter() - t) / reps
        random.seed(0)  # the winner's iteration (the drop-in returns inlier positions and F only)
        best, F, mask, _, _ = core.ransac_f8_pyrandom(x1, x2, H, 0.06, device=local_rank)
        out["host_sampling_ms"] = round(float(core.last_timings()[6]), 3)
        # the drop-in path's own GPU time (HIP events inside the call: the
        # chunked fits + scores, and the whole span to the select's end)
        core.set_call_timing(True)
        dk = []
        for _ in range(reps):
            random.seed(0)
            core.ransac_f8_pyrandom(x1, x2, H, 0.06, device=local_rank)
            tm = core.last_timings()
            dk.append((tm[3], tm[1]))
        core.set_call_timing(False)
        dropin_fit_score, dropin_span = (float(np.median([v[i] for v in dk])) for i in range(2))
        out["end_to_end_call"] = "GetInliersRANSAC(points1, points2, index, 0.06, n_max=H), the drop-in's whole call"
    else:
        h0, h1 = sfm_dist.hypothesis_range(H, world, rank)

        def one():
            random.seed(0)
            return sfm_dist.ransac_sharded(
                len(x1), H, rank, world,
                lambda a, b: core.ransac_f8_range(x1, x2, H, a, b, 0.06, device=local_rank)[:2],
                lambda k, M: core.ransac_combine(comm, k, M),
                lambda M: core.ransac_mask(x1, x2, M, 0.06, device=local_rank))
        for _ in range(3):
            one()
        if world > 1:
            torch.distributed.barrier()
        t = time.perf_counter()
        for _ in range(reps):
            best, F, mask = one()
        t_e2e = (time.perf_counter() - t) / reps
        if world > 1:
            t_t = torch.tensor([t_e2e], dtype=torch.float64)
            torch.distributed.all_reduce(t_t, op=torch.distributed.ReduceOp.MAX)
            t_e2e = float(t_t.item())
        out["sharding"] = f"hypotheses [{h0}, {h1}) on rank {rank} of {world}; packed-key max all-reduce (RCCL)"
        if rank == 0:  # the sharded result against the unsharded call on this GPU (same stream state)
            random.seed(0)
            b1, F1, m1 = core.ransac_f8_pyrandom(x1, x2, H, 0.06, device=local_rank)[:3]
            out["multi_rank_check"] = {
                "best_iter": [int(best), int(b1)], "F_equal": bool(F is not None and F1 is not None
                                                                     and np.array_equal(np.asarray(F), F1)),
                "mask_equal": bool(np.array_equal(np.asarray(mask, dtype=bool), np.asarray(m1, dtype=bool))),
                "ok": bool(int(best) == int(b1) and F is not None and F1 is not None
                           and np.array_equal(np.asarray(F), F1)
                           and np.array_equal(np.asarray(mask, dtype=bool), np.asarray(m1, dtype=bool)))}
    kt = []
    for _ in range(reps):
        core.ransac_f8(x1, x2, samples, 0.06, device=local_rank)
        tm = core.last_timings()
        kt.append((tm[1], tm[3], tm[4]))
    k_all, k_score, k_fit = (float(np.median([v[i] for v in kt])) for i in range(3))
    n = len(x1)
    score_flops = H * n * 50.0                       # ~50 fp64 flops per (hypothesis, corr.)
    all_flops = H * (n * 50.0 + 25e3)                # + ~25 kflop for each 8-point fit
    out.update({
        "hyps_per_s_end_to_end": round(H / t_e2e, 1),
        "hyps_per_s_kernels": round(H / (k_all * 1e-3), 1),
        "kernel_ms": round(k_all, 4), "score_kernel_ms": round(k_score, 4), "fit_kernel_ms": round(k_fit, 4),
        "best_iter": int(best), "inliers": int(np.count_nonzero(mask)),
        "fp64": {"bound": "valu-issue (ransac.roofline)", "score_tflops": round(score_flops / (k_score * 1e-3) / 1e12, 2),
                 "kernels_tflops": round(all_flops / (k_all * 1e-3) / 1e12, 2), "peak_tflops": FP64_PEAK_TFLOPS,
                 "score_frac": round(score_flops / (k_score * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
                 "formula": "score: H*N*50 flop; kernels: H*(N*50 + 25e3) flop (SURVEY §8(d)); algorithmic-equivalent: the score proves most pairs outliers with a packed float prefilter and runs the FP64 test only on the survivors, so it executes far fewer FP64 flops",
                 "score_bound": "VALU issue, not FP64: score_frac above 1 is an algorithmic-equivalent FP64 rate of mostly FP32 work, not a utilisation; the VALU-issue fraction is ransac.roofline"}})
    slots, src = ransac_valu_slots()
    if slots.get("oneshot"):  # the roofline that bounds the score: VALU issue, not FP64
        ach = slots["oneshot"] / (k_score * 1e-3)
        out["roofline"] = {"kernel": "k_epi_score (one-shot, 16,384 hypotheses x 5,000 pairs)", "bound": "valu-issue",
                           "achieved": round(ach / 1e9, 1), "peak": round(VALU_SLOTS_PEAK / 1e9, 1),
                           "unit": "G VALU issue slots/s (wave64, 2 SIMD cycles each)",
                           "frac": round(ach / VALU_SLOTS_PEAK, 4), "traffic": None,
                           "source": src, "time": "the score kernel's HIP events, this run"}
    if comm is None:  # the drop-in call's own kernels (timed above)
        if slots.get("dropin") and "roofline" in out:
            ach = slots["dropin"] / (dropin_fit_score * 1e-3)
            out["roofline"].update({"dropin_achieved": round(ach / 1e9, 1),
                                    "dropin_frac": round(ach / VALU_SLOTS_PEAK, 4),
                                    "dropin_note": "the drop-in call's chunked fits + scores (first fit to last "
                                                   "score, HIP events), executed slots from the PMC passes"})
        out["fp64"].update({
            "dropin_fit_score_ms": round(dropin_fit_score, 4), "dropin_span_ms": round(dropin_span, 4),
            "dropin_tflops": round(all_flops / (dropin_fit_score * 1e-3) / 1e12, 2),
            "dropin_frac": round(all_flops / (dropin_fit_score * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
            "dropin_note": "the drop-in path's own fits + scores (chunked, in-call sampling; HIP events from the "
                           "first fit to the last score), not the one-shot given-table launch"})
    return out, (x1, x2, samples)


def ba_leg(workload, args, world, rank, local_rank, comm, barrier, allmax):
    """One BA workload: the converged solve (RMSE), W warmup + K timed LM
    iterations from x0 (barrier + synchronize around, max over ranks), and a
    second run of the same K iterations with HIP events on for the per-phase
    split (each event record costs the stream a few us, so the timed run has
    none).  Every rank builds the same problem and keeps its point shard."""
    prob = syn.ba_problem_cfg(workload, dense=False)
    cams0 = np.column_stack([prob["rotvec0"], np.einsum("nij,nj->ni", -prob["R0"], prob["C0"])])
    ci, pi, ob, X0, (lo, hi) = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"],
                                                 world, rank)
    ba = core.BAProblem(cams0, X0, ci, pi, ob, K, comm=comm, device=local_rank)
    ba.reset()
    conv = ba.solve(max_iterations=100)
    conv_c, conv_x = ba.download() if world > 1 else (None, None)
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
    ba.reset()
    ba.set_timing(True)
    ba.solve(max_iterations=args.steps, fixed_iterations=True)
    ktimes = ba.kernel_times()
    ba.set_timing(False)
    ba.close()
    check = None
    if world > 1:
        # multi-GPU correctness on the driver's node (after the timed region):
        # every rank must hold the same converged cost, and rank 0 re-solves
        # the whole problem alone on its GPU -- the sharded solve must take
        # the same LM path (iterations, accepted steps) to the same cost, its
        # shard's points and the cameras as close as the multi-rank tests ask
        spread = allmax(conv["cost"]) + allmax(-conv["cost"])
        if rank == 0:
            one = core.BAProblem(cams0, prob["X0"], prob["cam_idx"], prob["pt_idx"], prob["obs"], K,
                                 device=local_rank)
            srep = one.solve(max_iterations=100)
            s_c, s_x = one.download()
            one.close()
            dx = float(np.abs(conv_x - s_x[lo:hi]).max()) if hi > lo else 0.0
            dc = float(np.abs(conv_c - s_c).max())
            check = {"ranks": world, "cost_spread_over_ranks": spread,
                     "sharded": {"iterations": conv["iterations"], "accepted": conv["accepted"], "cost": conv["cost"]},
                     "single_rank": {"iterations": srep["iterations"], "accepted": srep["accepted"],
                                     "cost": srep["cost"]},
                     "max_abs_diff_points_rank0_shard": dx, "max_abs_diff_cameras": dc,
                     "ok": bool(spread == 0.0 and conv["iterations"] == srep["iterations"]
                                and conv["accepted"] == srep["accepted"]
                                and abs(conv["cost"] - srep["cost"]) <= 1e-9 * abs(srep["cost"])
                                and dx < 1e-6 and dc < 1e-8),
                     "tolerance": "same iterations and accepted steps, cost within 1e-9 relative, points 1e-6 and "
                                  "cameras 1e-8 absolute (the in-process multi-rank tests' bounds)"}
        barrier()
    return dict(workload=workload, prob=prob, cams0=cams0, dt=dt, rep=rep, conv=conv, ktimes=ktimes,
                hi=hi, n_obs_local=len(ci), n_pts_local=len(X0), check=check)


def ba_record(leg, args, world):
    """The bench-line fields of one BA leg (value, roofline, fp64, per-kernel
    split, step mix, RMSE)."""
    prob, workload = leg["prob"], leg["workload"]
    n_obs_total, n_pts_total = len(prob["cam_idx"]), prob["n_pts"]
    n_pairs = n_pairs_of(prob["pt_idx"][prob["pt_idx"] < leg["hi"]] if world > 1 else prob["pt_idx"])
    ns = 6 * prob["n_cams"]
    nblocks = prob["n_cams"] * (prob["n_cams"] + 1) // 2
    ms_per_step = leg["dt"] / args.steps * 1e3
    # roofline of the LM iteration: compulsory bytes of the
    # minimal three-pass design, B_iter = 52 N_obs + 240 N_pts, against the
    # measured time of an iteration (ms_per_step)
    iter_bytes = 52 * n_obs_total + 240 * n_pts_total
    ach = iter_bytes / (ms_per_step * 1e-3) / 1e9
    pmc, pmc_src = pmc_iteration(workload) if world == 1 else ({}, None)
    roof = {"kernel": "LM iteration (all kernels of one damped solve + trial evaluation)", "bound": "hbm",
            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
            "traffic": int(sum(pmc.values())) if pmc else None, "algorithmic_bytes": int(iter_bytes),
            "formula": "52*N_obs + 240*N_pts per iteration (SURVEY §8(d)), / ms_per_step",
            "traffic_source": (f"{pmc_src} (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE passes of tools/ba_once.py "
                               f"{workload}; (2*FETCH+WRITE) KiB summed over the kernels / iterations)")
            if pmc else None}
    flops = ba_flops(prob["pt_idx"], prob["n_cams"])
    kern = {}
    for k, v in leg["ktimes"].items():
        e = {"ms": round(v, 4)}
        d = design_bytes(k, leg["n_obs_local"], leg["n_pts_local"], n_pairs, nblocks, ns)
        if d is not None:
            e["design_bytes"] = int(d)
            e["design_GBs"] = round(d / (v * 1e-3) / 1e9, 1) if v > 0 else None
        if k == "cholesky":
            e["flops"] = ns ** 3 / 3
            e["tflops"] = round(ns ** 3 / 3 / (v * 1e-3) / 1e12, 4) if v > 0 else None
            e["note"] = "reduced camera solve: persistent block Gauss-Jordan (one launch); flops = n^3/3 (Cholesky)"
        kern[k] = e
    conv, rep = leg["conv"], leg["rep"]
    return {
        "value": round(args.steps / leg["dt"], 3),
        "unit": "LM-iterations/s",
        "ms_per_step": round(ms_per_step, 4),
        "workload": f"{workload}: BA {prob['n_cams']} cams / {n_pts_total} pts / {n_obs_total} obs, "
                    f"Schur-complement LM, points sharded over {world} rank(s)",
        "roofline": roof,
        "fp64": {"flops_per_iteration": flops, "achieved_tflops": round(flops / (ms_per_step * 1e-3) / 1e12, 3),
                 "peak_tflops": FP64_PEAK_TFLOPS,
                 "frac": round(flops / (ms_per_step * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 5),
                 "formula": "400 N_obs + sum_p(108 k_p + 216 k_p(k_p+1)/2) + (6 n_c)^3/3 (SURVEY §8(d))"},
        "kernels_ms_per_iter": kern,
        "pmc_bytes_per_iter": {k: int(v) for k, v in pmc.items()} if pmc else None,
        "step_mix": {"timed_steps": args.steps, "accepted": rep["accepted"],
                     "note": "fixed iterations from x0; the problem converges in ~5, later steps are rejected "
                             "(a rejected step skips k_linearize / the camera blocks)",
                     "converged_solve": {"iterations": conv["iterations"], "accepted": conv["accepted"],
                                         "loop_ms": round(conv["t_loop_ms"], 3),
                                         "ms_per_iteration": round(conv["t_loop_ms"] / max(1, conv["iterations"]), 4)}},
        "converged_LM_it_per_s": round(conv["iterations"] / (conv["t_loop_ms"] * 1e-3), 2) if conv["t_loop_ms"] else None,
        **({"multi_rank_check": leg["check"]} if leg.get("check") else {}),
        "rmse": {f"{workload}_initial": round(syn.rmse_from_cost(conv["cost0"], n_obs_total), 6),
                 f"{workload}_gpu": round(syn.rmse_from_cost(conv["cost"], n_obs_total), 6),
                 "lm_iterations": conv["iterations"]},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg5", choices=["cfg3", "cfg4", "cfg5"],
                    help="headline BA workload (value); cfg5 is BASELINE's scaling config")
    ap.add_argument("--no-secondary", action="store_true", help="skip the cfg4 (north-star) sub-record")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ransac-hyps", type=int, default=16384)
    ap.add_argument("--force-comm", action="store_true", help="use the RCCL communicator even with one rank")
    ap.add_argument("--no-next-rows", action="store_true", help="skip the SURVEY §8(f) row measurements")
    ap.add_argument("--no-end-to-end", action="store_true", help="skip the dense perform_bundle_adjustment call")
    ap.add_argument("--no-shard-local", action="store_true", help="skip the per-rank shard bound")
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

    comm = None
    if world > 1 or args.force_comm:
        uid = [core.Comm.unique_id() if rank == 0 else None]
        if world > 1:
            torch.distributed.broadcast_object_list(uid, src=0)
        comm = core.Comm(uid[0], world, rank, device=local_rank)

    # ---------------- BA: the headline workload, then the cfg4 sub-record
    legs = [ba_leg(args.workload, args, world, rank, local_rank, comm, barrier, allmax)]
    second = None if args.no_secondary else ("cfg4" if args.workload != "cfg4" else None)
    if second:
        legs.append(ba_leg(second, args, world, rank, local_rank, comm, barrier, allmax))

    # ---------------- the drop-in end to end, and the per-rank shard bound (N = 1 only)
    e2e, shards = {}, None
    if world == 1 and not args.no_end_to_end:
        for wl in [args.workload] + ([second] if second else []):
            e2e[wl] = end_to_end_ba(wl)
    if world == 1 and not args.no_shard_local:
        shards = shard_local(args.workload, args.steps, args.warmup)

    # ---------------- RANSAC (config 2)
    ransac, (x1, x2, samples) = ransac_leg(args, world, rank, local_rank, comm)
    if comm is not None:
        comm.close()

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    head = ba_record(legs[0], args, world)
    out = {
        "metric": "BA LM-iterations/sec (+ RANSAC hypotheses/sec, final reproj RMSE vs ref)",
        "value": head["value"],
        "unit": "LM-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (sfm_synthetic.ba_problem, seed 3)",
        "config": {"workload": head["workload"],
                   "parallelism": f"point-shard x{world} + RCCL all-reduce of the reduced camera system"},
        "roofline": head["roofline"],
        "fp64": head["fp64"],
        "kernels_ms_per_iter": head["kernels_ms_per_iter"],
        "pmc_bytes_per_iter": head["pmc_bytes_per_iter"],
        "step_mix": head["step_mix"],
        "converged_LM_it_per_s": head["converged_LM_it_per_s"],
        **({"multi_rank_check": head["multi_rank_check"]} if "multi_rank_check" in head else {}),
        "rmse": head["rmse"],
        "ransac": ransac,
    }
    if second:
        out[second] = ba_record(legs[1], args, world)
    if args.workload in e2e:
        out["end_to_end"] = e2e[args.workload]
    if second in e2e:
        out[second]["end_to_end"] = e2e[second]
    if shards:
        out["shard_local"] = shards
    if world == 1:
        out["rmse"].update(cfg3_rmse_vs_reference())
    cpu_leg = world == 1 and not args.no_cpu_baseline
    if cpu_leg:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        # the OpenMP legs: threads pinned to cores, packed (read at the
        # runtime's first parallel region, i.e. after this)
        os.environ.setdefault("OMP_PROC_BIND", "close")
        os.environ.setdefault("OMP_PLACES", "cores")
    if not args.no_next_rows:
        out["next_rows"] = next_rows(core, local_rank, cpu_leg)
    if cpu_leg:
        import oracle as O  # test infrastructure: the CPU restatement, timed as the baseline
        avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        sweep = sorted({t for t in (1, 4, 16, 64, 128) if t <= avail} | {min(128, avail)})
        cpu = {}
        for i, leg in enumerate(legs):
            rec = out if i == 0 else out[leg["workload"]]
            base = cpu_baseline_ba(leg["prob"], leg["cams0"], sweep, single=leg["workload"] != "cfg5")
            best_t = max(base["strong"], key=lambda t: base["strong"][t][0])
            sv, srep, sdt = base["strong"][best_t]
            n_obs_total = len(leg["prob"]["cam_idx"])
            if "oracle" in base:
                rec["rmse"][f"{leg['workload']}_oracle"] = round(syn.rmse_from_cost(base["oracle"][1]["cost"], n_obs_total), 6)
            cpu[leg["workload"]] = {
                "value": round(sv, 4), "unit": "LM-iterations/s", "cores": best_t, "kind": "port",
                "sample": f"CPU-strong OpenMP Schur-LM (oracle/sfm_cpu_strong.c), full {leg['workload']} problem, "
                          f"{srep['iterations']} LM iterations to convergence in {sdt:.2f}s on {best_t} threads "
                          f"(the fastest of the thread sweep)",
                "speedup": round(rec["value"] / sv, 1),
                "thread_sweep": {str(t): {"LM_it_per_s": round(v[0], 4), "s": round(v[2], 3)}
                                 for t, v in sorted(base["strong"].items())},
                "reference_extrapolated": base["ref"]}
            if "converged" in base:
                cv, crep, cdt, ct = base["converged"]
                cpu[leg["workload"]]["converged_at_fastest_threads"] = {
                    "LM_it_per_s": round(cv, 4), "threads": ct, "iterations": crep["iterations"],
                    "s": round(cdt, 3), "status": crep.get("status")}
            if "oracle" in base:
                ov, orep, odt = base["oracle"]
                cpu[leg["workload"]]["single_thread_oracle"] = {
                    "value": round(ov, 4), "unit": "LM-iterations/s", "cores": 1,
                    "sample": f"C Schur-LM (oracle/sfm_oracle.c), {orep['iterations']} iterations in {odt:.2f}s"}
        rv, rdt, rth = cpu_baseline_ransac(x1, x2, samples, sweep)
        c1 = cpu_cfg1()
        head_cpu = cpu[args.workload]
        out["cpu_baseline"] = dict(head_cpu)
        if second:
            out[second]["cpu_baseline"] = cpu[second]
        out["cpu_baseline"].update({
            "cfg3_as_shipped": cpu_cfg3_as_shipped(),
            "ransac_cfg2": {"hyps_per_s": round(rv, 1), "cores": rth,
                            "sample": f"OpenMP RANSAC (sfm_cpu_strong.c cs_ransac: hypotheses split over {rth} "
                                      f"threads, same counts as the oracle), all {len(samples)} cfg2 hypotheses in "
                                      f"{rdt:.2f}s"},
            "ransac_cfg1": c1,
            "cpu": _cpu_model(), "os_cpu_count": os.cpu_count(), "cpus_available_to_this_process": avail,
            "physical_cores": _physical_cores(),
            "threads_note": "thread counts beyond the CPUs this process may use are not run; the sweep's "
                            "fastest point is the baseline",
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
            "OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"), "OMP_PLACES": os.environ.get("OMP_PLACES"),
            "OPENBLAS_NUM_THREADS": os.environ.get("OPENBLAS_NUM_THREADS")})
    print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


def cfg3_rmse_vs_reference():
    """cfg3 (6 cams / 2000 pts / 10k obs, seed 3) solved on the GPU against the
    reference's converged least-squares oracle (tests/golden/ba.npz, scipy
    trf on the reference residual, captured by importing the reference)."""
    p = syn.ba_problem(6, 2000, 5, seed=3, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    c, X, r = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=100)
    res = core.ba_residuals(c, X, p["cam_idx"], p["pt_idx"], p["obs"], K)
    n = len(p["cam_idx"])
    g = np.load(os.path.join(REPO, "tests", "golden", "ba.npz"))
    return {"cfg3_gpu": round(syn.rmse_from_cost(0.5 * float(res @ res), n), 6),
            "cfg3_reference_converged": round(syn.rmse_from_cost(float(g["cfg3_cost_conv"]), n), 6),
            "cfg3_initial": round(syn.rmse_from_cost(float(g["cfg3_cost0"]), n), 6)}


def cpu_cfg1():
    """cfg1: P3Data pair 1_2 after the homography step (N = 558), 1000
    hypotheses, seed 0 (tests/golden/ransac_p3data.npz): the GPU drop-in call
    and the C oracle on the same table."""
    import oracle as O
    p = np.load(os.path.join(REPO, "tests", "golden", "ransac_p3data.npz"))
    key = "s0_1_2"
    x1, x2 = p[key + "_x1"], p[key + "_x2"]
    st = (3, tuple(int(v) for v in p[key + "_state_before"]), None)
    random.setstate(st)
    table = core.sample_table(len(x1), 8, 1000)
    random.setstate(st)
    core.ransac_f8_pyrandom(x1, x2, 1000, 0.06)
    random.setstate(st)
    t = time.perf_counter()
    core.ransac_f8_pyrandom(x1, x2, 1000, 0.06)
    tg = time.perf_counter() - t
    t = time.perf_counter()
    O.ransac(x1, x2, table, 0.06)
    tc = time.perf_counter() - t
    return {"N": int(len(x1)), "hypotheses": 1000, "gpu_call_ms": round(tg * 1e3, 3),
            "cpu_oracle_ms": round(tc * 1e3, 3), "cpu_threads": 1}


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
