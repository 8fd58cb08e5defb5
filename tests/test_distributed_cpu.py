"""World-size-2 `gloo` tests of the multi-GPU partitioning on CPU.

The GPU path (csrc/ba.hip + sfm_dist.py) shards points -- with all their
observations -- across ranks and sums the ranks' partial reduced camera
systems with one all-reduce per LM iteration.  Here a numpy restatement of
that partial system (test infrastructure, built on the oracle's residual)
runs on two gloo ranks and must equal the single-process system; a full
distributed LM loop must reproduce the single-process oracle's converged
cost.  RANSAC hypothesis sharding runs sfm_dist.ransac_sharded with the
packed-key combine over gloo and must give the unsharded winner, model and
mask.  LinearTriangulation point ranges (sfm_dist.triangulate_sharded) and
the image-pair spread (sfm_dist.pair_loop_spread: homography chain and F
tables replicated, F-RANSACs round-robin) are gathered over gloo and must
equal the single-process results and random-stream state.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
import sfm_dist
import sfm_synthetic as syn

K = syn.K_REF
H_RANSAC = 601  # odd: uneven shards


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def linearize(R, t, X, cam, pt, obs):
    """r, Jc (n,2,6), Jp (n,2,3) with the left-perturbation model of csrc/ba.hip."""
    p = np.einsum("nij,nj->ni", R[cam], X[pt])
    xc = p + t[cam]
    u = xc @ K.T
    iw = 1.0 / (u[:, 2] + 1e-8)
    pu, pv = u[:, 0] * iw, u[:, 1] * iw
    r = np.column_stack([obs[:, 0] - pu, obs[:, 1] - pv])
    A = np.empty((len(cam), 2, 3))
    A[:, 0, :] = -(iw[:, None] * K[0] - (pu * iw)[:, None] * K[2])
    A[:, 1, :] = -(iw[:, None] * K[1] - (pv * iw)[:, None] * K[2])
    px = np.zeros((len(cam), 3, 3))  # -[p]x
    px[:, 0, 1], px[:, 0, 2] = p[:, 2], -p[:, 1]
    px[:, 1, 0], px[:, 1, 2] = -p[:, 2], p[:, 0]
    px[:, 2, 0], px[:, 2, 1] = p[:, 1], -p[:, 0]
    Jc = np.concatenate([A @ px, A], axis=2)
    Jp = A @ R[cam]
    return r, Jc, Jp


def partial_system(R, t, X, cam, pt, obs, nc, lam):
    """The payload one rank contributes: S_undamped, diag(U), g_c, sum Z q, cost, + per-point pieces."""
    r, Jc, Jp = linearize(R, t, X, cam, pt, obs)
    npt = len(X)
    V = np.zeros((npt, 3, 3))
    np.add.at(V, pt, np.einsum("nai,naj->nij", Jp, Jp))
    gp = np.zeros((npt, 3))
    np.add.at(gp, pt, np.einsum("nai,na->ni", Jp, r))
    dV = np.diagonal(V, axis1=1, axis2=2)
    Vd = V + lam * np.einsum("ni,ij->nij", np.clip(dV, 1e-6, 1e32), np.eye(3))
    Vi = np.linalg.inv(Vd)
    W = np.einsum("nai,naj->nij", Jc, Jp)  # 6x3
    ns = 6 * nc
    S = np.zeros((ns, ns))
    U = np.einsum("nai,naj->nij", Jc, Jc)
    for o in range(len(cam)):
        c = cam[o]
        S[6 * c:6 * c + 6, 6 * c:6 * c + 6] += U[o]
    gc = np.zeros(ns)
    np.add.at(gc.reshape(nc, 6), cam, np.einsum("nai,na->ni", Jc, r))
    bZ = np.zeros(ns)
    Vg = np.einsum("nij,nj->ni", Vi, gp)
    np.add.at(bZ.reshape(nc, 6), cam, np.einsum("nij,nj->ni", W, Vg[pt]))
    # -W V^-1 W^T over co-observing pairs
    order = np.argsort(pt, kind="stable")
    starts = np.searchsorted(pt[order], np.arange(npt + 1))
    for q in range(npt):
        os_ = order[starts[q]:starts[q + 1]]
        Y = np.einsum("aij,jk->aik", W[os_], Vi[q])
        for ia, a in enumerate(os_):
            for b in os_:
                ca, cb = cam[a], cam[b]
                S[6 * ca:6 * ca + 6, 6 * cb:6 * cb + 6] -= Y[ia] @ W[b].T
    Ud = np.zeros((nc, 6))
    np.add.at(Ud, cam, np.diagonal(U, axis1=1, axis2=2))
    diagU = Ud.ravel()
    cost = 0.5 * float((r ** 2).sum())
    return dict(S=S, diagU=diagU, gc=gc, bZ=bZ, cost=cost, V=V, gp=gp, Vi=Vi, W=W, Jc=Jc, Jp=Jp)


# stand-ins with the reference's RNG use (GetHomographyInliers.py:124-126,
# GetInliersRANSAC.py:53-55) and the oracle as the fit/score
N_PAIR_ITERS = 60


def _tri_inputs():
    _, _, _, m = syn.two_view(n=301, seed=5)
    return m["clean1"], m["clean2"]


def _tri_fn(a, b):
    _, _, _, m = syn.two_view(n=301, seed=5)
    return O.triangulate(syn.K_REF, np.zeros(3), np.eye(3), m["C2"], m["R2"], a, b)


def _pair_inputs():
    pairs, pts = [], []
    for k, n in enumerate((150, 7, 120, 90)):  # pair 1 has too few matches for any draw
        a, b, _, _ = syn.two_view(n=n, seed=20 + k)
        pairs.append((a, b, np.arange(n, dtype=np.int64) * 3 + k))
        pts.append((a, b))
    return pairs, (lambda k, h_idx: (pts[k][0][(h_idx - k) // 3], pts[k][1][(h_idx - k) // 3]))


def _homography(x1, x2, index):
    n = len(x1)
    if n < 4:
        return None, np.array([])
    table = np.array([random.sample(range(n), 4) for _ in range(N_PAIR_ITERS)], dtype=np.int32)
    b, _, Hm, m = O.ransac_h(x1, x2, table, 30.0)
    return (Hm, index[m]) if b >= 0 else (None, np.array([], dtype=np.int64))


def _draw_f_table(n, n_iter):
    return np.array([random.sample(range(n), 8) for _ in range(n_iter)], dtype=np.int32)


def _f_ransac(p1, p2, h_idx, table):
    if table is None:
        return None, np.array([])
    b, _, F, m = O.ransac(p1, p2, table, 0.06)
    return (F, h_idx[m]) if b >= 0 else (None, np.array([]))


def _pair_loop_sequential():
    """The reference driver's order: homography RANSAC, then F-RANSAC, pair by pair."""
    random.seed(11)
    pairs, f_points = _pair_inputs()
    out = []
    for k, (x1, x2, index) in enumerate(pairs):
        Hm, h_idx = _homography(x1, x2, index)
        p1, p2 = f_points(k, h_idx)
        table = _draw_f_table(len(p1), N_PAIR_ITERS) if len(p1) >= 8 else None
        out.append((Hm, h_idx) + _f_ransac(p1, p2, h_idx, table))
    return out, random.getstate()


def _rank_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prob = syn.ba_problem(4, 120, 3, seed=9, dense=False)
        R = prob["R0"]
        t = np.einsum("nij,nj->ni", -R, prob["C0"])
        ci, pi, ob, X0, _ = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"], world, rank)
        part = partial_system(R, t, X0, ci, pi, ob, 4, 1e-3)
        payload = torch.from_numpy(np.concatenate([part["S"].ravel(), part["diagU"], part["gc"], part["bZ"],
                                                   [part["cost"]]]))
        dist.all_reduce(payload)
        # RANSAC: the real sharding code (sfm_dist.ransac_sharded + the
        # torch.distributed key combine) with the oracle as each shard's
        # fit/score (on the GPU: sfm_ransac_f8_pyrandom_range)
        x1, x2, _, _ = syn.two_view(n=400, seed=4)
        random.seed(7)
        table = np.array([random.sample(range(400), 8) for _ in range(H_RANSAC)], dtype=np.int32)
        st_after = random.getstate()

        def shard_fn(h0, h1):
            if h1 <= h0:
                return 0, np.zeros(9)
            b, counts, F, _ = O.ransac(x1, x2, table[h0:h1], 0.06)
            return (sfm_dist.shard_key(counts[b], h0 + b), F) if b >= 0 else (0, np.zeros(9))

        it, F, mask = sfm_dist.ransac_sharded(len(x1), H_RANSAC, rank, world, shard_fn,
                                              sfm_dist.combine_keys_torch, lambda M: O.ransac_mask(x1, x2, M, 0.06))
        # LinearTriangulation over point ranges, gathered over gloo
        Xt = sfm_dist.triangulate_sharded(_tri_fn, *_tri_inputs(), world, rank, sfm_dist.allgather_torch)
        # image pairs: the homography chain and the F tables on every rank,
        # the F-RANSACs round-robin, the results gathered over gloo
        random.seed(11)
        spread = sfm_dist.pair_loop_spread(*_pair_inputs(), world, rank, _homography, _draw_f_table, _f_ransac,
                                           sfm_dist.allgather_torch, n_max=N_PAIR_ITERS)
        q.put((rank, payload.numpy(), (it, F, mask, st_after), Xt, (spread, random.getstate())))
    finally:
        dist.destroy_process_group()


def test_sharded_reduced_system_equals_full_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    prob = syn.ba_problem(4, 120, 3, seed=9, dense=False)
    R = prob["R0"]
    t = np.einsum("nij,nj->ni", -R, prob["C0"])
    full = partial_system(R, t, prob["X0"], prob["cam_idx"], prob["pt_idx"], prob["obs"], 4, 1e-3)
    ref = np.concatenate([full["S"].ravel(), full["diagU"], full["gc"], full["bZ"], [full["cost"]]])
    # the unsharded RANSAC on the same table
    x1, x2, _, _ = syn.two_view(n=400, seed=4)
    random.seed(7)
    table = np.array([random.sample(range(400), 8) for _ in range(H_RANSAC)], dtype=np.int32)
    st_ref = random.getstate()
    b_ref, _, F_ref, mask_ref = O.ransac(x1, x2, table, 0.06)
    assert b_ref >= 0
    X_ref = _tri_fn(*_tri_inputs())
    seq, st_seq = _pair_loop_sequential()
    assert any(r[2] is not None for r in seq) and seq[1][2] is None
    for rank, payload, (it, F, mask, st_after), Xt, (spread, st_spread) in out:
        assert np.allclose(payload, ref, rtol=1e-10, atol=1e-9 * np.abs(ref).max())
        assert it == b_ref and np.array_equal(F, F_ref) and np.array_equal(mask, mask_ref)
        assert st_after == st_ref  # every rank's stream ends where the unsharded draw leaves it
        assert np.array_equal(Xt, X_ref)
        assert st_spread == st_seq  # every rank's stream ends where the sequential loop leaves it
        assert len(spread) == len(seq)
        for (H1, h1, F1, f1), (H2, h2, F2, f2) in zip(spread, seq):
            assert (H1 is None) == (H2 is None) and (H1 is None or np.array_equal(H1, H2))
            assert np.array_equal(h1, h2) and np.array_equal(f1, f2)
            assert (F1 is None) == (F2 is None) and (F1 is None or np.array_equal(F1, F2))


def distributed_lm(shards, nc, iters=30, lam=1e-4):
    """The control flow of sfm_ba_solve (csrc/ba.hip) over in-memory shards;
    `sum` stands for the all-reduce.  Returns the final global cost."""
    Rs = [s["R"].copy() for s in shards]
    ts = [s["t"].copy() for s in shards]
    Xs = [s["X"].copy() for s in shards]
    ns = 6 * nc
    nu = 2.0
    cost = None
    for _ in range(iters):
        parts = [partial_system(Rs[k], ts[k], Xs[k], s["cam"], s["pt"], s["obs"], nc, lam)
                 for k, s in enumerate(shards)]
        S = sum(p["S"] for p in parts)
        diagU = sum(p["diagU"] for p in parts)
        gc = sum(p["gc"] for p in parts)
        bZ = sum(p["bZ"] for p in parts)
        if cost is None:
            cost = sum(p["cost"] for p in parts)
        S = S + np.diag(lam * np.clip(diagU, 1e-6, 1e32))
        dc = np.linalg.solve(S, -gc + bZ)
        model = float(dc @ (lam * np.clip(diagU, 1e-6, 1e32) * dc - gc))
        new_cost = 0.0
        trial = []
        for k, (s, p) in enumerate(zip(shards, parts)):
            # -g_p - sum_o W_o^T dc  (accumulated per point)
            acc = -p["gp"].copy()
            np.add.at(acc, s["pt"], -np.einsum("nij,ni->nj", p["W"], dc.reshape(nc, 6)[s["cam"]]))
            dp = np.einsum("nij,nj->ni", p["Vi"], acc)
            dV = np.diagonal(p["V"], axis1=1, axis2=2)
            model += float((dp * (lam * np.clip(dV, 1e-6, 1e32) * dp - p["gp"])).sum())
            dR = np.stack([O.rotvec_to_R(w) for w in dc.reshape(nc, 6)[:, :3]])
            Rn = np.einsum("nij,njk->nik", dR, Rs[k])
            tn = ts[k] + dc.reshape(nc, 6)[:, 3:]
            Xn = Xs[k] + dp
            r, _, _ = linearize(Rn, tn, Xn, s["cam"], s["pt"], s["obs"])
            new_cost += 0.5 * float((r ** 2).sum())
            trial.append((Rn, tn, Xn))
        model *= 0.5
        rho = (cost - new_cost) / model if model > 0 else -1
        if rho > 1e-3:
            for k, (Rn, tn, Xn) in enumerate(trial):
                Rs[k], ts[k], Xs[k] = Rn, tn, Xn
            f = 1 - (2 * rho - 1) ** 3
            lam *= max(f, 1 / 3)
            nu = 2.0
            if cost - new_cost < 1e-10 * new_cost:
                cost = new_cost
                break
            cost = new_cost
        else:
            lam *= nu
            nu *= 2
    return cost


@pytest.mark.parametrize("world", [1, 2, 3])
def test_distributed_lm_matches_single_process_oracle(world):
    prob = syn.ba_problem(4, 120, 3, seed=9, dense=False)
    R = prob["R0"]
    t = np.einsum("nij,nj->ni", -R, prob["C0"])
    shards = []
    for rank in range(world):
        ci, pi, ob, X0, _ = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"], world, rank)
        shards.append(dict(R=R, t=t, X=X0, cam=ci, pt=pi, obs=ob))
    cost = distributed_lm(shards, 4)
    cams0 = np.column_stack([prob["rotvec0"], t])
    _, _, rep = O.ba_lm(cams0, prob["X0"], prob["cam_idx"], prob["pt_idx"], prob["obs"], K)
    assert abs(cost - rep["cost"]) <= 1e-6 * rep["cost"]


def test_shard_covers_every_observation_once():
    prob = syn.ba_problem(7, 1001, 4, seed=2, dense=False)
    seen = []
    for world in (1, 2, 3, 8):
        tot = 0
        for rank in range(world):
            ci, pi, ob, X0, (lo, hi) = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"],
                                                        world, rank)
            assert len(X0) == hi - lo and (len(pi) == 0 or (pi.min() >= 0 and pi.max() < hi - lo))
            tot += len(ci)
        seen.append(tot)
    assert all(s == len(prob["cam_idx"]) for s in seen)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_combine_keys_keeps_first_strict_max(world):
    """The packed key's max over any split of the hypotheses equals the
    reference's scan: max count, earliest iteration on ties; key 0 when no
    hypothesis has an inlier."""
    rng = np.random.default_rng(world)
    for counts in (rng.integers(0, 5, 997), np.zeros(50, dtype=int), np.array([3, 7, 7, 1, 7])):
        H = len(counts)
        keys = []
        for rank in range(world):
            h0, h1 = sfm_dist.hypothesis_range(H, world, rank)
            c = counts[h0:h1]
            keys.append(sfm_dist.shard_key(c.max(), h0 + int(np.argmax(c))) if len(c) else 0)
        cnt, it = sfm_dist.key_iter(max(keys))
        best, best_i = 0, -1
        for i, c in enumerate(counts):  # GetInliersRANSAC.py:85-88
            if c > best:
                best, best_i = c, i
        assert (cnt, it) == (best, best_i)
