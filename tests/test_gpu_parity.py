"""Parity of the HIP path (through the C-ABI and the drop-in modules) with the
reference, on a real MI355X.  Expected values come from tests/golden/ (made
by importing the reference, tests/golden/make_golden.py) and from the C
oracle (oracle/sfm_oracle.c) on the same seeded inputs.

Tolerances:
  * RANSAC: identical per-hypothesis counts, best iteration, inlier set,
    and the global random state afterwards; |F - F_ref| / |F_ref| <= 1e-9.
  * 8-point F and DLT triangulation: relative error <= 1e-9.
  * BA: reprojection RMSE within 1e-4 (relative) of the converged
    least-squares solution of the reference residual, and never above the
    as-shipped reference result.
"""
import random

import numpy as np
import pytest

import oracle as O
import sfm_synthetic as syn

pytestmark = pytest.mark.gpu
K = syn.K_REF


@pytest.fixture(scope="module")
def core():
    import _sfmcore
    _sfmcore.require_device()
    return _sfmcore


def rel(a, b):
    return np.abs(np.asarray(a) - np.asarray(b)).max() / np.abs(np.asarray(b)).max()


def degenerate_samples(x1, x2, samples):
    rows = np.concatenate([x1[samples], x2[samples]], axis=2)
    return np.array([len(np.unique(r, axis=0)) < len(r) for r in rows])


# ------------------------------------------------------------------ F / RANSAC
def test_f8_batch_matches_reference(core, golden):
    g = golden("f8.npz")
    F = core.f8_batch(g["p1"], g["p2"])
    r = np.abs(F - g["F"]).max(axis=(1, 2)) / np.abs(g["F"]).max(axis=(1, 2))
    assert r.max() < 1e-9, r.max()


@pytest.mark.parametrize("n", [9, 20, 100, 558])
def test_estimate_fundamental_matrix_general_n(core, golden, n):
    from EstimateFundamentalMatrix import EstimateFundamentalMatrix
    g = golden("f8.npz")
    F = EstimateFundamentalMatrix(g[f"genN{n}_p1"], g[f"genN{n}_p2"])
    assert rel(F, g[f"genN{n}_F"]) < 1e-9


def test_estimate_fundamental_matrix_8pt_dropin(core, golden):
    from EstimateFundamentalMatrix import EstimateFundamentalMatrix
    g = golden("f8.npz")
    for i in range(0, 512, 97):
        assert rel(EstimateFundamentalMatrix(g["p1"][i].tolist(), g["p2"][i]), g["F"][i]) < 1e-9
    with pytest.raises(ValueError):
        EstimateFundamentalMatrix(np.zeros((8, 3)), np.zeros((8, 3)))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ransac_cfg2_bit_exact(core, golden, seed):
    """cfg2: N=5000, 40 % outliers, 16384 (seed 0) / 2000 hypotheses."""
    from GetInliersRANSAC import GetInliersRANSAC
    c = golden("ransac_cfg2.npz")
    x1, x2, idx = c["x1"], c["x2"], c["index"]
    H = int(c[f"s{seed}_n_max"])
    random.seed(seed)
    st = random.getstate()
    samples = np.array([random.sample(range(len(x1)), 8) for _ in range(H)], dtype=np.int32)
    best, F, mask, counts = core.ransac_f8(x1, x2, samples, 0.06, want_counts=True)
    assert np.array_equal(counts, c[f"s{seed}_counts"].astype(np.int32))
    assert best == int(c[f"s{seed}_best_iter"])
    # through the drop-in, consuming the global random stream itself
    random.setstate(st)
    inl, outl, F2 = GetInliersRANSAC(x1, x2, idx, 0.06, H)
    assert np.array_equal(inl, c[f"s{seed}_inlier_pos"])
    assert np.array_equal(np.sort(np.concatenate([inl, outl])), idx)
    assert rel(F2, c[f"s{seed}_F"]) < 1e-9
    assert np.array_equal(np.array(random.getstate()[1], dtype=np.uint32), c[f"s{seed}_state_after"])


@pytest.mark.parametrize("seed", [0, 1])
def test_ransac_p3data_all_pairs(core, golden, seed):
    """cfg1: the reference driver's 10 image pairs (Wrapper_dev.py:69-123)."""
    from GetInliersRANSAC import get_inliers_ransac
    p = golden("ransac_p3data.npz")
    n_pairs = 0
    for a in range(1, 6):
        for b in range(a + 1, 6):
            key = f"s{seed}_{a}_{b}"
            if key + "_x1" not in p:
                continue
            random.setstate((3, tuple(int(v) for v in p[key + "_state_before"]), None))
            F, f_idx = get_inliers_ransac(p[key + "_x1"], p[key + "_x2"], p[key + "_index"], threshold=0.06,
                                          n_max=1000)
            assert np.array_equal(np.asarray(f_idx, dtype=np.int64), p[key + "_inlier_idx"]), key
            assert rel(F, p[key + "_F"]) < 1e-9, key
            assert np.array_equal(np.array(random.getstate()[1], dtype=np.uint32), p[key + "_state_after"])
            n_pairs += 1
    assert n_pairs == 10


def test_ransac_p3data_pair12_counts(core, golden):
    p = golden("ransac_p3data.npz")
    key = "s0_1_2"
    x1, x2 = p[key + "_x1"], p[key + "_x2"]
    random.setstate((3, tuple(int(v) for v in p[key + "_state_before"]), None))
    samples = core.sample_table(len(x1), 8, 1000)
    best, F, mask, counts = core.ransac_f8(x1, x2, samples, 0.06, want_counts=True)
    degen = degenerate_samples(x1, x2, samples)
    assert np.array_equal(counts[~degen], p[key + "_counts"][~degen])
    assert best == int(np.argmax(p[key + "_counts"]))
    assert np.array_equal(p[key + "_index"][mask], p[key + "_inlier_idx"])


def test_ransac_matches_oracle_random_inputs(core):
    rng = np.random.default_rng(7)
    for N, H in ((8, 50), (64, 300), (1000, 700), (4097, 129)):
        x1, x2, _, _ = syn.two_view(n=N, seed=int(rng.integers(1 << 30)))
        samples = np.stack([rng.choice(N, 8, replace=False) for _ in range(H)]).astype(np.int32)
        b, counts, F, mask = O.ransac(x1, x2, samples, 0.5)
        b2, F2, mask2, counts2 = core.ransac_f8(x1, x2, samples, 0.5, want_counts=True)
        assert np.array_equal(counts, counts2)
        assert b == b2
        if b >= 0:
            assert np.array_equal(mask, mask2)
            assert rel(F2, F) < 1e-9


@pytest.mark.parametrize("H", [1, 7, 2048, 5000])
def test_ransac_pyrandom_matches_host_table(core, H):
    """In-call sampling (chunked MT19937 replay pipelined with the GPU work)
    draws exactly sample_table's table, gives the same counts / winner /
    mask, and leaves the global random stream where sample_table leaves it."""
    x1, x2, _, _ = syn.two_view(n=3000, seed=4)
    for run, (tbl_fn, pyr_fn, kk, thr) in enumerate([(core.ransac_f8, core.ransac_f8_pyrandom, 8, 0.06),
                                                     (core.ransac_h4, core.ransac_h4_pyrandom, 4, 30.0)]):
        random.seed(100 + H + run)
        samples = core.sample_table(3000, kk, H)
        st_ref = random.getstate()
        b0, M0, m0, c0 = tbl_fn(x1, x2, samples, thr, want_counts=True)
        random.seed(100 + H + run)
        b1, M1, m1, c1, s1 = pyr_fn(x1, x2, H, thr, want_counts=True, want_samples=True)
        assert random.getstate() == st_ref
        assert np.array_equal(s1, samples)
        assert np.array_equal(c1, c0) and b1 == b0 and np.array_equal(m1, m0)
        if b0 >= 0:
            assert np.array_equal(M1, M0)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_ransac_sharded_matches_single_rank_cfg2(core, golden, world):
    """Hypothesis-sharded F-RANSAC on cfg2 (16384 hypotheses):
    every rank draws the whole table from the global stream and scores its
    range (sfm_ransac_f8_pyrandom_range); the keys are combined across
    `world` in-process ranks sharing the GPU (sfm_ransac_combine, one host
    thread per rank); the winner's F gives the mask.  Counts, winner, F,
    mask and the RNG state equal the unsharded reference fixture."""
    import threading
    import sfm_dist
    c = golden("ransac_cfg2.npz")
    x1, x2 = c["x1"], c["x2"]
    H = int(c["s0_n_max"])
    shards, counts = [], []
    for rank in range(world):  # each rank's own process would do exactly this
        random.seed(0)
        h0, h1 = sfm_dist.hypothesis_range(H, world, rank)
        key, F, cnt = core.ransac_f8_range(x1, x2, H, h0, h1, 0.06, want_counts=True)
        assert np.array_equal(np.array(random.getstate()[1], dtype=np.uint32), c["s0_state_after"])
        shards.append((key, F))
        counts.append(cnt)
    assert np.array_equal(np.concatenate(counts), c["s0_counts"].astype(np.int32))
    comms = core.local_group(world)
    out = [None] * world

    def run(rank):
        out[rank] = sfm_dist.ransac_sharded(
            len(x1), H, rank, world, lambda h0, h1: shards[rank],
            lambda k, M: core.ransac_combine(comms[rank], k, M),
            lambda M: core.ransac_mask(x1, x2, M, 0.06))

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    for cm in comms:
        cm.close()
    for it, F, mask in out:
        assert it == int(c["s0_best_iter"])
        assert rel(F, c["s0_F"]) < 1e-9
        assert np.array_equal(np.nonzero(mask)[0], c["s0_inlier_pos"])
    # the given-table form agrees shard by shard
    random.seed(0)
    table = core.sample_table(len(x1), 8, H)
    for rank in range(world):
        h0, h1 = sfm_dist.hypothesis_range(H, world, rank)
        k2, F2, _ = core.ransac_f8_range(x1, x2, H, h0, h1, 0.06, samples=table)
        assert k2 == shards[rank][0] and (k2 == 0 or np.array_equal(F2, shards[rank][1]))


def test_ransac_h4_sharded_matches_single_rank(core):
    """Homography shards: concatenated counts and the combined key equal the
    unsharded in-call RANSAC's."""
    import sfm_dist
    x1, x2, _, _ = syn.two_view(n=3000, seed=4)
    random.seed(11)
    b0, M0, m0, c0, _ = core.ransac_h4_pyrandom(x1, x2, 3001, 30.0, want_counts=True)
    keys, cnts = [], []
    for rank in range(3):
        random.seed(11)
        h0, h1 = sfm_dist.hypothesis_range(3001, 3, rank)
        k, M, cnt = core.ransac_h4_range(x1, x2, 3001, h0, h1, 30.0, want_counts=True)
        keys.append((k, M))
        cnts.append(cnt)
    assert np.array_equal(np.concatenate(cnts), c0)
    k, M = max(keys, key=lambda km: km[0])
    assert sfm_dist.key_iter(k)[1] == b0 and np.array_equal(M, M0)
    assert np.array_equal(core.ransac_mask(x1, x2, M, 30.0, model=4), m0)


def test_ransac_edge_cases(core):
    from GetInliersRANSAC import GetInliersRANSAC, get_inliers_ransac
    x1, x2, idx, _ = syn.two_view(n=200, seed=3)
    # N < 8: early exit, random untouched
    random.seed(5)
    st = random.getstate()
    inl, outl, F = GetInliersRANSAC(x1[:7], x2[:7], idx[:7])
    assert len(inl) == 0 and F is None and np.array_equal(outl, idx[:7]) and random.getstate() == st
    # n_max = 0: no hypotheses
    inl, outl, F = GetInliersRANSAC(x1, x2, idx, 0.06, 0)
    assert F is None and len(inl) == 0
    # threshold 0: every count is 0 -> None, but the stream still advanced n_max draws
    random.seed(5)
    Fb, fi = get_inliers_ransac(x1, x2, idx, threshold=0.0, n_max=37)
    st_after = random.getstate()
    random.seed(5)
    for _ in range(37):
        random.sample(range(200), 8)
    assert Fb is None and fi.dtype == np.float64 and len(fi) == 0 and random.getstate() == st_after
    # NaN correspondence: hypotheses that sample it score 0, others unaffected
    y1 = x1.copy()
    y1[3] = np.nan
    rng = np.random.default_rng(1)
    samples = np.stack([rng.choice(200, 8, replace=False) for _ in range(200)]).astype(np.int32)
    b, counts, _, _ = O.ransac(y1, x2, samples, 0.5)
    b2, _, _, counts2 = core.ransac_f8(y1, x2, samples, 0.5, want_counts=True)
    assert np.array_equal(counts, counts2) and b == b2
    # points that are not (N, 2) (Phase 1/GetInliersRANSAC.py:49-50, each
    # iteration's EstimateFundamentalMatrix raising at :80-81 inside the
    # loop's try): n_max draws consumed, (np.array([]), index, None) back;
    # N mismatched between the two sets: np.hstack raises before any draw.
    # The device call after them continues the same stream (tests/test_abi.py
    # covers the shapes without a device)
    random.seed(9)
    inl, outl, F = GetInliersRANSAC(np.hstack([x1, np.ones((200, 1))]), x2, idx, 0.06, 40)
    assert F is None and inl.shape == (0,) and np.array_equal(outl, idx)
    st_dev = random.getstate()
    random.seed(9)
    for _ in range(40):
        random.sample(range(200), 8)
    assert random.getstate() == st_dev
    with pytest.raises(ValueError):
        GetInliersRANSAC(x1, x2[:150], idx, 0.06, 40)
    assert random.getstate() == st_dev
    Fd, fd = get_inliers_ransac(x1, x2, idx, threshold=0.06, n_max=64)
    st_after = random.getstate()
    random.setstate(st_dev)
    samples = np.array([random.sample(range(200), 8) for _ in range(64)], dtype=np.int32)
    assert random.getstate() == st_after
    b, counts, Fo, mo = O.ransac(x1, x2, samples, 0.06)
    assert b >= 0 and rel(Fd, Fo) < 1e-9 and np.array_equal(np.asarray(fd, dtype=np.int64), idx[mo])


def test_ransac_full_size_properties(core):
    """cfg2 at 4x the hypotheses: every reported inlier satisfies the test,
    the winner's count equals its mask size and is the maximum."""
    x1, x2, idx, _ = syn.two_view(n=5000, seed=9)
    random.seed(11)
    samples = core.sample_table(5000, 8, 65536)
    best, F, mask, counts = core.ransac_f8(x1, x2, samples, 0.06, want_counts=True)
    assert counts.max() == counts[best] == mask.sum()
    assert np.argmax(counts) == best
    assert np.array_equal(O.ransac_mask(x1, x2, F, 0.06), mask)


# ------------------------------------------------------------- triangulation
def test_triangulation_matches_reference(core, golden):
    from LinearTriangulation import LinearTriangulation, linear_triangulation
    t = golden("triangulation.npz")
    for i in range(4):
        X = linear_triangulation(K, np.zeros(3), np.eye(3), t["p3_Cset"][i], t["p3_Rset"][i], t["p3_x1"], t["p3_x2"])
        assert rel(X, t[f"p3_X{i}"]) < 1e-9
    X = LinearTriangulation(K, np.zeros(3), np.eye(3), t["syn_C2"], t["syn_R2"], t["syn_x1"], t["syn_x2"])
    r = np.abs(X - t["syn_X"]).max(axis=1) / np.abs(t["syn_X"]).max(axis=1)
    assert r.max() < 1e-9
    assert LinearTriangulation(K, np.zeros(3), np.eye(3), t["syn_C2"], t["syn_R2"], [], []).shape == (0,)


def test_triangulation_large_vs_oracle(core):
    _, _, _, m = syn.two_view(n=200_000, seed=4)
    rng = np.random.default_rng(2)
    x1 = m["clean1"] + rng.normal(0, 0.5, m["clean1"].shape)
    x2 = m["clean2"] + rng.normal(0, 0.5, m["clean2"].shape)
    P1 = O.projection(K, np.zeros(3), np.eye(3))
    P2 = O.projection(K, m["C2"], m["R2"])
    X = core.triangulate(P1, P2, x1, x2)
    Xo = O.triangulate(K, np.zeros(3), np.eye(3), m["C2"], m["R2"], x1[:20000], x2[:20000])
    r = np.abs(X[:20000] - Xo).max(axis=1) / np.abs(Xo).max(axis=1)
    assert r.max() < 1e-9
    # size-independent property: the DLT point reprojects close to the data
    err = np.abs(core.project(P2, X) - x2).max()
    assert err < 5.0


def test_nonlinear_triangulation_bit_exact_vs_reference(core, golden):
    """One GPU thread per point runs MINPACK lmdif: identical to the
    reference's per-point scipy 'lm' on every fixture row (P3Data poses,
    cfg2 inliers, outliers that stop at max_nfev, x0-kept rows)."""
    from NonLinearTriangulation import NonLinearTriangulation, nonlinear_triangulation
    t, g = golden("triangulation.npz"), golden("nltri.npz")
    for i in range(4):
        X = nonlinear_triangulation(K, np.zeros(3), np.eye(3), t["p3_Cset"][i], t["p3_Rset"][i], t["p3_x1"],
                                    t["p3_x2"], t[f"p3_X{i}"])
        assert np.array_equal(X, g[f"p3_X{i}"]), i
    X = NonLinearTriangulation(K, np.zeros(3), np.eye(3), t["syn_C2"], t["syn_R2"], t["syn_x1"], t["syn_x2"],
                               t["syn_X"])
    assert np.array_equal(X, g["syn_X"])
    with np.errstate(all="ignore"):
        X = NonLinearTriangulation(K, np.zeros(3), np.eye(3), g["out_C2"], g["out_R2"], g["out_x1"], g["out_x2"],
                                   g["out_X0"])
    assert np.array_equal(X, g["out_X"], equal_nan=True)
    assert NonLinearTriangulation(K, np.zeros(3), np.eye(3), t["syn_C2"], t["syn_R2"], [], [], []).shape == (0,)


def test_nonlinear_triangulation_large_vs_oracle(core):
    """200k noisy points with 20 % outliers: GPU == oracle bit for bit on a
    20k slice (the oracle's budget) and per-point info codes agree; the
    refined points never reproject worse than the DLT start."""
    x1, x2, _, m = syn.two_view(n=200_000, seed=7, outlier_frac=0.2)
    P1 = O.projection(K, np.zeros(3), np.eye(3))
    P2 = O.projection(K, m["C2"], m["R2"])
    X0 = core.triangulate(P1, P2, x1, x2)
    X, info = core.triangulate_nonlinear(P1, P2, x1, x2, X0, max_nfev=50)
    Xo, info_o = O.nltri(K, np.zeros(3), np.eye(3), m["C2"], m["R2"], x1[:20000], x2[:20000], X0[:20000])
    assert np.array_equal(X[:20000], Xo, equal_nan=True)
    assert np.array_equal(info[:20000], info_o)

    def cost(Xs, sel):
        Xh = np.column_stack([Xs, np.ones(len(Xs))])
        c = 0
        for P, x in ((P1, x1[sel]), (P2, x2[sel])):
            h = Xh @ P.T
            c = c + ((x - h[:, :2] / h[:, 2:3]) ** 2).sum(1)
        return c
    ok = info > 0
    assert ok.mean() > 0.99
    assert np.all(cost(X[ok], ok) <= cost(X0[ok], ok) * (1 + 1e-9) + 1e-12)


# --------------------------------------------------------------- homography
def _set_state(st):
    random.setstate((3, tuple(int(v) for v in st), None))


def _state_array():
    return np.array(random.getstate()[1], dtype=np.uint64).astype(np.uint32)


def test_find_homography_matches_reference(core, golden):
    from GetHomographyInliers import find_homography
    g = golden("homography.npz")
    Hs = core.h4_batch(g["f4_p1"], g["f4_p2"])
    r = np.abs(Hs - g["f4_H"]).max(axis=(1, 2)) / np.abs(g["f4_H"]).max(axis=(1, 2))
    assert r.max() < 1e-9
    for n in (4, 5, 9, 64, 1000):
        assert rel(find_homography(g[f"fN{n}_p1"], g[f"fN{n}_p2"]), g[f"fN{n}_H"]) < 1e-9
    with pytest.raises(ValueError):
        find_homography(np.zeros((3, 2)), np.zeros((3, 2)))


@pytest.mark.parametrize("key,H", [("s0_1_2", 1000), ("plane", 4096), ("cfg2", 2000)])
def test_homography_ransac_counts_bit_exact(core, golden, key, H):
    g = golden("homography.npz")
    x1, x2 = g[key + "_x1"], g[key + "_x2"]
    _set_state(g[key + "_state_before"])
    samples = core.sample_table(len(x1), 4, H)
    assert np.array_equal(_state_array(), g[key + "_state_after"])
    best, Hb, mask, counts = core.ransac_h4(x1, x2, samples, 30.0, want_counts=True)
    assert np.array_equal(counts, g[key + "_counts"])
    assert best == int(np.argmax(g[key + "_counts"]))
    assert rel(Hb, g[key + "_H"]) < 1e-9


@pytest.mark.parametrize("seed", [0, 1])
def test_p3data_pair_loop_homography_then_f(core, golden, seed):
    """The driver's pair loop (Wrapper_dev.py:67-123) through the drop-ins:
    homography RANSAC then F-RANSAC on its inliers, for all 10 pairs, with
    one global random stream.  Every H, H-inlier set, MT state, F and
    F-inlier set equals the reference's."""
    from GetHomographyInliers import get_homography_inliers
    from GetInliersRANSAC import get_inliers_ransac
    from itertools import combinations
    g, p = golden("homography.npz"), golden("ransac_p3data.npz")
    fx, fy = p["feature_x"], p["feature_y"]
    random.seed(seed)
    for (a, b) in combinations(range(1, 6), 2):
        key = f"s{seed}_{a}_{b}"
        assert np.array_equal(_state_array(), g[key + "_state_before"]), key
        H, h_idx = get_homography_inliers(g[key + "_x1"], g[key + "_x2"], g[key + "_index"], threshold=30,
                                          n_max=1000)
        assert np.array_equal(_state_array(), g[key + "_state_after"]), key
        assert rel(H, g[key + "_H"]) < 1e-9, key
        assert np.array_equal(h_idx, g[key + "_inlier_idx"]), key
        i1 = np.hstack((fx[h_idx, a - 1].reshape((-1, 1)), fy[h_idx, a - 1].reshape((-1, 1))))
        i2 = np.hstack((fx[h_idx, b - 1].reshape((-1, 1)), fy[h_idx, b - 1].reshape((-1, 1))))
        F, f_idx = get_inliers_ransac(i1, i2, h_idx, threshold=0.06, n_max=1000)
        assert np.array_equal(_state_array(), p[key + "_state_after"]), key
        assert np.array_equal(np.asarray(f_idx, dtype=np.int64), p[key + "_inlier_idx"]), key


@pytest.mark.parametrize("world", [1, 2, 3])
def test_p3data_pair_loop_spread_over_ranks(core, golden, world):
    """Image-pair spreading (sfm_dist.pair_loop_spread): every
    rank replays the homography chain and draws every F table on the global
    stream, then scores its round-robin share of the 10 F-RANSACs from the
    drawn tables.  Ranks run one after another here (each from the same
    seed, as separate processes would); every rank's stream ends where the
    reference's sequential loop leaves it, and the merged H / F inlier sets
    equal the reference's (Wrapper_dev.py:67-123)."""
    import functools
    import sfm_dist
    from GetHomographyInliers import get_homography_inliers
    from itertools import combinations
    g, p = golden("homography.npz"), golden("ransac_p3data.npz")
    fx, fy = p["feature_x"], p["feature_y"]
    seed = 0
    keys = [f"s{seed}_{a}_{b}" for (a, b) in combinations(range(1, 6), 2)]
    ab = list(combinations(range(1, 6), 2))
    pairs = [(g[k + "_x1"], g[k + "_x2"], g[k + "_index"]) for k in keys]

    def f_points(k, h_idx):
        a, b = ab[k]
        return (np.hstack((fx[h_idx, a - 1].reshape((-1, 1)), fy[h_idx, a - 1].reshape((-1, 1)))),
                np.hstack((fx[h_idx, b - 1].reshape((-1, 1)), fy[h_idx, b - 1].reshape((-1, 1)))))

    homography = functools.partial(get_homography_inliers, threshold=30, n_max=1000)
    f_ransac = functools.partial(sfm_dist.f_ransac_from_table, core, threshold=0.06)
    plans, parts = [], []
    for rank in range(world):
        random.seed(seed)
        plan = sfm_dist.pair_loop_plan(pairs, f_points, homography, lambda n, it: core.sample_table(n, 8, it))
        assert np.array_equal(_state_array(), p[keys[-1] + "_state_after"])
        plans.append(plan)
        parts.append(sfm_dist.pair_loop_local(plan, world, rank, f_ransac))
    assert sorted(k for part in parts for k in part) == list(range(len(pairs)))
    for rank in range(world):
        out = sfm_dist.pair_loop_merge(plans[rank], parts)
        for k, (H, h_idx, F, f_idx) in zip(keys, out):
            assert rel(H, g[k + "_H"]) < 1e-9, k
            assert np.array_equal(h_idx, g[k + "_inlier_idx"]), k
            assert np.array_equal(np.asarray(f_idx, dtype=np.int64), p[k + "_inlier_idx"]), k


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_triangulation_sharded_equals_whole(core, world):
    """LinearTriangulation over contiguous point ranges (sfm_dist.
    triangulate_sharded): the ranges gathered in rank order are bitwise the
    single call's result (points are independent)."""
    import sfm_dist
    _, _, _, m = syn.two_view(n=20_001, seed=6)
    x1, x2 = m["clean1"], m["clean2"]
    P1 = O.projection(K, np.zeros(3), np.eye(3))
    P2 = O.projection(K, m["C2"], m["R2"])
    whole = core.triangulate(P1, P2, x1, x2)
    pieces = [None] * world

    def tri(a, b):
        return core.triangulate(P1, P2, a, b)

    for rank in range(world):  # the gather returns the pieces computed so far; the last rank sees all
        lo, hi = sfm_dist.point_shard(len(x1), world, rank)
        pieces[rank] = tri(x1[lo:hi], x2[lo:hi])
    X = sfm_dist.triangulate_sharded(tri, x1, x2, world, world - 1,
                                     lambda mine: [pc if r < world - 1 else mine for r, pc in enumerate(pieces)])
    assert np.array_equal(X, whole)


def test_homography_ransac_edge_cases(core):
    from GetHomographyInliers import get_homography_inliers
    random.seed(3)
    st = random.getstate()
    H, inl = get_homography_inliers(np.zeros((3, 2)), np.zeros((3, 2)), np.arange(3))
    assert H is None and len(inl) == 0 and random.getstate() == st  # no draw below 4 points
    x1, x2, _, _ = syn.two_view(n=300, seed=2)
    H, inl = get_homography_inliers(x1, x2, np.arange(300), threshold=0, n_max=50)
    assert H is None and len(inl) == 0  # strict '<' against 0 never holds
    H, inl = get_homography_inliers(x1, x2, np.arange(300), n_max=0)
    assert H is None and len(inl) == 0
    # ties: duplicated hypotheses keep the earliest
    random.seed(5)
    samples = core.sample_table(300, 4, 64)
    samples = np.concatenate([samples, samples])
    best, _, _, counts = core.ransac_h4(x1, x2, samples, 30.0, want_counts=True)
    assert best == int(np.argmax(counts)) and best < 64


def test_homography_ransac_large_vs_oracle(core):
    """N = 200k points, 2048 hypotheses: counts equal the oracle's on every
    hypothesis (the oracle sweeps all N), and the winner's mask reproduces
    its count."""
    x1, x2, _, _ = syn.two_view(n=200_000, seed=9, outlier_frac=0.3)
    random.seed(9)
    samples = core.sample_table(len(x1), 4, 2048)
    best, Hb, mask, counts = core.ransac_h4(x1, x2, samples, 30.0, want_counts=True)
    Hs = core.h4_batch(x1[samples[:256]], x2[samples[:256]])
    assert np.array_equal(counts[:256], O.h_score(x1, x2, Hs, 30.0))
    assert mask.sum() == counts[best] == counts.max()


# ---------------------------------------------------------------------- PnP
def test_linear_pnp_matches_reference(core, golden):
    from LinearPnP import LinearPnP
    g = golden("pnp.npz")
    well = agree = 0
    for X, x, C, R in zip(g["lp4_X"], g["lp4_x"], g["lp4_C"], g["lp4_R"]):
        c, r, br = core.linear_pnp(X, x, K)
        co, ro, bro = O.linear_pnp(X, x, K)
        assert br == bro
        if br == 0:  # well-defined branch: the reference's pose
            well += 1
            assert np.abs(c - C).max() <= 1e-9 * max(1.0, np.abs(C).max())
            assert np.abs(r - R).max() <= 1e-9
        else:
            agree += np.abs(r - ro).max() < 1e-6
    assert well >= 256
    for n in (5, 6, 10, 100, 500):
        C, R = LinearPnP(g[f"lpN{n}_X"], g[f"lpN{n}_x"], K)
        if core.linear_pnp(g[f"lpN{n}_X"], g[f"lpN{n}_x"], K)[2] == 0:
            assert np.abs(C - g[f"lpN{n}_C"]).max() <= 1e-9 * max(1.0, np.abs(g[f"lpN{n}_C"]).max()), n
            assert np.abs(R - g[f"lpN{n}_R"]).max() <= 1e-9, n
    with pytest.raises(ValueError):
        LinearPnP(np.zeros((3, 3)), np.zeros((3, 2)), K)


@pytest.mark.parametrize("name", ["o30_t200", "o30_t8", "o60_t4"])
@pytest.mark.parametrize("seed", [0, 1])
def test_pnp_ransac_matches_reference(core, golden, name, seed):
    """PnPRANSAC through the drop-in: the global random stream, the winner
    and the final pose equal the reference's; per-hypothesis counts equal on
    every well-defined hypothesis."""
    from PnPRANSAC import PnPRANSAC
    g = golden("pnp.npz")
    X, x, thr = g[name + "_X"], g[name + "_x"], float(g[name + "_thr"])
    key = f"{name}_s{seed}"
    ref_counts = g[key + "_counts"]
    _set_state(g[key + "_state_before"])
    C, R = PnPRANSAC(X, x, K, threshold=thr, n_max=len(ref_counts))
    assert np.array_equal(_state_array(), g[key + "_state_after"])
    assert np.abs(C - g[key + "_C"]).max() <= 1e-9 * max(1.0, np.abs(g[key + "_C"]).max())
    assert np.abs(R - g[key + "_R"]).max() <= 1e-9
    _set_state(g[key + "_state_before"])
    samples = core.sample_table(len(X), 4, len(ref_counts))
    best, bc, _, _, counts, branches = core.pnp_ransac(X, x, K, samples, thr, want_counts=True)
    well = branches == 0
    assert np.array_equal(counts[well], ref_counts[well])
    assert best == int(np.argmax(ref_counts)) and bc == ref_counts.max()


def test_pnp_ransac_fallback_and_edges(core, capsys):
    from PnPRANSAC import PnPRANSAC
    X, x, _, _ = _pnp_scene(300, 3)
    random.seed(4)
    C, R = PnPRANSAC(X, x, K, threshold=1e-12, n_max=20)  # no hypothesis reaches 4 inliers
    assert "Warning: PnP RANSAC failed, using linear PnP on all points" in capsys.readouterr().out
    Co, Ro, br = O.linear_pnp(X, x, K)
    assert core.linear_pnp(X, x, K)[2] == br
    if br == 0:  # the det(R) < 0 branch is LAPACK-noise defined
        assert np.abs(C - Co).max() <= 1e-8 * np.abs(Co).max() and np.abs(R - Ro).max() <= 1e-8
    assert np.abs(R @ R.T - np.eye(3)).max() < 1e-12 and np.linalg.det(R) > 0
    with pytest.raises(ValueError):
        PnPRANSAC(X[:3], x[:3], K)


def _pnp_scene(n, seed, outlier_frac=0.0):
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(5, 12, n)])
    R = syn.rotvec_to_matrix([0.02, -0.15, 0.01])[0]
    C = np.array([1.0, 0.05, 0.1])
    u = (K @ (R @ (X - C).T)).T
    x = u[:, :2] / u[:, 2:3] + rng.normal(0, 0.5, (n, 2))
    k = int(round(outlier_frac * n))
    if k:
        o = rng.choice(n, k, replace=False)
        x[o] = np.column_stack([rng.uniform(0, 1280, k), rng.uniform(0, 960, k)])
    return X, x, C, R


def test_nonlinear_pnp_matches_reference(core, golden, capsys):
    """Device sin/cos are not correctly rounded and the m-long reductions
    run in parallel, so the GPU lmdif is not bit-identical: it stops at the
    same minimum (cost within 1e-9 relative of the reference's) with the pose
    within 1e-5 (ftol-terminated LM pins flat directions only that far)."""
    from NonlinearPnP import NonLinearPnPLoss, nonlinear_PnP
    from scipy.spatial.transform import Rotation
    g = golden("pnp.npz")

    def cost(C, R, X, x):
        p = np.hstack([Rotation.from_matrix(R).as_rotvec(), -R @ C])
        r = NonLinearPnPLoss(p, X, x, K)
        return 0.5 * r @ r
    for name in ("clean50", "clean2000", "out500", "tiny3", "four"):
        k = "nl_" + name
        C, R = nonlinear_PnP(K, g[k + "_C0"], g[k + "_R0"], g[k + "_x"], g[k + "_X"])
        assert np.abs(C - g[k + "_C"]).max() <= 1e-5 * max(1.0, np.abs(g[k + "_C"]).max()), name
        assert np.abs(R - g[k + "_R"]).max() <= 1e-5, name
        if len(g[k + "_X"]) >= 4:
            cg, cr = cost(C, R, g[k + "_X"], g[k + "_x"]), cost(g[k + "_C"], g[k + "_R"], g[k + "_X"], g[k + "_x"])
            assert abs(cg - cr) <= 1e-9 * cr + 1e-12, name
    # the reference's except path: non-finite start -> inputs back, message printed
    X, x, C0, R0 = _pnp_scene(50, 2)
    C, R = nonlinear_PnP(K, np.array([np.nan, 0, 0]), R0, x, X)
    assert np.isnan(C[0]) and np.array_equal(R, R0)
    assert "Non-linear PnP optimization failed" in capsys.readouterr().out


def test_pnp_large_vs_oracle(core):
    """100k points, 30 % outliers: RANSAC winner / counts vs the oracle on
    the well-defined hypotheses, then NonlinearPnP from the winner."""
    X, x, Ct, Rt = _pnp_scene(100_000, 11, outlier_frac=0.3)
    random.seed(11)
    samples = core.sample_table(len(X), 4, 512)
    best, bc, C, R, counts, branches = core.pnp_ransac(X, x, K, samples, 8.0, want_counts=True)
    ob, oc, obr, oC, oR = O.pnp_ransac(X, x, K, samples, 8.0)
    well = (branches == 0) & (obr == 0)
    assert np.array_equal(counts[well], oc[well])
    assert best == ob or branches[best] == 1 or obr[ob] == 1
    Cn, Rn, info = core.nonlinear_pnp(X[:20000], x[:20000], K, C, R)
    Co, Ro, info_o = O.nonlinear_pnp(X[:20000], x[:20000], K, C, R)
    assert info > 0 and np.abs(Cn - Co).max() <= 1e-6 * max(1.0, np.abs(Co).max())


def _ill_pnp_scene(n, kind, eps, seed):
    rng = np.random.default_rng(seed)
    t = rng.uniform(-2, 2, n)
    if kind == "line":  # near-collinear: the rotation about the line is (almost) unobservable
        X = np.column_stack([t, 0.5 * t, 8 + 0.3 * t]) + eps * rng.standard_normal((n, 3))
    elif kind == "plane":  # near-planar
        X = np.column_stack([t, rng.uniform(-2, 2, n), np.full(n, 8.0)]) + eps * rng.standard_normal((n, 3))
    else:  # one point repeated: a rank-deficient Jacobian
        X = np.tile([[0.3, -0.2, 8.0]], (n, 1))
    R = syn.rotvec_to_matrix([0.02, -0.15, 0.01])[0]
    C = np.array([1.0, 0.05, 0.1])
    h = (K @ (R @ (X - C).T)).T
    x = h[:, :2] / h[:, 2:3] + rng.normal(0, 0.5, (n, 2))
    return X, x, C + 0.05, syn.rotvec_to_matrix([0.03, -0.14, 0.0])[0]


def _pnp_cost(X, x, C, R):
    h = (K @ (R @ (X - C).T)).T
    r = x - h[:, :2] / (h[:, 2:3] + 1e-8)
    return float((r * r).sum())


@pytest.mark.parametrize("n", [4, 5, 6])
@pytest.mark.parametrize("eps", [1e-3, 1e-6, 1e-9])
@pytest.mark.parametrize("kind", ["plane", "line"])
def test_nonlinear_pnp_ill_conditioned_vs_oracle(core, kind, eps, n):
    """NonlinearPnP (NonlinearPnP.py:97-123) on near-planar and near-collinear
    point sets of 4..6 points, against the oracle's lmdif (MINPACK's
    Householder qrfac on J).  The device factors J by CholeskyQR2 (shifted
    CholeskyQR3 when the Gram factor needs a shift, reported in info's flags).
    Near-planar: the same minimum, pose within 2e-5 (lmdif's ftol-level
    flat directions, as for the well-conditioned fixtures).  Near-collinear:
    the rotation about the line is unobservable, so the poses may differ
    along it; the cost reached agrees within 1e-3 relative and the stop
    reason is the same."""
    X, x, C0, R0 = _ill_pnp_scene(n, kind, eps, n)
    Cg, Rg, ig, fl = core.nonlinear_pnp(X, x, K, C0, R0, want_flags=True)
    Co, Ro, io = O.nonlinear_pnp(X, x, K, C0, R0)
    assert ig == io and fl in (0, 1, 3)
    cg, co = _pnp_cost(X, x, Cg, Rg), _pnp_cost(X, x, Co, Ro)
    if kind == "plane":
        assert np.abs(Cg - Co).max() <= 2e-5 and np.abs(Rg - Ro).max() <= 2e-5
        assert abs(cg - co) <= 1e-7 * co
    else:
        assert abs(cg - co) <= 1e-3 * co, (cg, co)


@pytest.mark.parametrize("wgs", [1, 2, 5, 16, 64])
@pytest.mark.parametrize("n,outl", [(5000, 0.3), (20000, 0.0), (7, 0.0)])
def test_nonlinear_pnp_workgroups_vs_oracle(core, monkeypatch, wgs, n, outl):
    """NonlinearPnP (NonlinearPnP.py:97-123) with the rows cut over `wgs`
    workgroups (every workgroup runs lmdif on all-gathered sums; n = 7 with
    64 workgroups leaves most slices empty): the same stop reason as the
    oracle's lmdif, pose within 1e-5, cost within 1e-9 relative -- the bar of
    the one-workgroup kernel."""
    X, x, C, R = _pnp_scene(n, 31, outl)
    C0 = C + 0.05
    R0 = syn.rotvec_to_matrix([0.03, -0.13, 0.02])[0]
    monkeypatch.setenv("SFM_NLPNP_WGS", str(wgs))
    Cg, Rg, ig = core.nonlinear_pnp(X, x, K, C0, R0)
    Co, Ro, io = O.nonlinear_pnp(X, x, K, C0, R0)
    assert ig == io
    assert np.abs(Cg - Co).max() <= 1e-5 * max(1.0, np.abs(Co).max()) and np.abs(Rg - Ro).max() <= 1e-5
    cg, co = _pnp_cost(X, x, Cg, Rg), _pnp_cost(X, x, Co, Ro)
    assert abs(cg - co) <= 1e-9 * co + 1e-12


def test_nonlinear_pnp_timeout_retry_equals_one_workgroup(core, monkeypatch):
    """A cross-workgroup hand-off that times out (forced by
    SFM_NLPNP_FORCE_TIMEOUT=1: every workgroup of the 8-workgroup launch
    aborts at its first hand-off) makes the host re-run the solve on one
    workgroup: the result is bitwise the one-workgroup solve's."""
    X, x, C, R = _pnp_scene(8000, 33, 0.2)
    C0 = C + 0.05
    R0 = syn.rotvec_to_matrix([0.03, -0.13, 0.02])[0]
    monkeypatch.setenv("SFM_NLPNP_WGS", "1")
    C1, R1, i1 = core.nonlinear_pnp(X, x, K, C0, R0)
    monkeypatch.setenv("SFM_NLPNP_WGS", "8")
    monkeypatch.setenv("SFM_NLPNP_FORCE_TIMEOUT", "1")
    Cr, Rr, ir = core.nonlinear_pnp(X, x, K, C0, R0)
    assert ir == i1 and np.array_equal(Cr, C1) and np.array_equal(Rr, R1)
    monkeypatch.delenv("SFM_NLPNP_FORCE_TIMEOUT")
    # and the 8-workgroup solve itself still runs: deterministic, and at the
    # one-workgroup minimum to the device NonlinearPnP's parity (DESIGN §3:
    # the row sums' order differs, so the iterates part at rounding level;
    # measured: 1.5e-7 on this pose's C)
    C8, R8, i8 = core.nonlinear_pnp(X, x, K, C0, R0)
    C8b, R8b, i8b = core.nonlinear_pnp(X, x, K, C0, R0)
    assert i8b == i8 and np.array_equal(C8b, C8) and np.array_equal(R8b, R8)
    assert i8 == i1 and np.abs(C8 - C1).max() <= 1e-5 * max(1.0, np.abs(C1).max()) and np.abs(R8 - R1).max() <= 1e-5
    c8, c1 = _pnp_cost(X, x, C8, R8), _pnp_cost(X, x, C1, R1)
    assert abs(c8 - c1) <= 1e-9 * c1 + 1e-12


def test_nonlinear_pnp_rank_deficient_flags(core):
    """A rank-deficient Jacobian (one point repeated): the Gram factor needs
    the shift, the third CholeskyQR pass runs and the flags say so; lmdif
    still ends with finite parameters no worse than the start."""
    X, x, C0, R0 = _ill_pnp_scene(5, "point", 0.0, 3)
    Cg, Rg, ig, fl = core.nonlinear_pnp(X, x, K, C0, R0, want_flags=True)
    assert fl & 1
    assert np.all(np.isfinite(Cg)) and np.all(np.isfinite(Rg))
    assert _pnp_cost(X, x, Cg, Rg) <= _pnp_cost(X, x, C0, R0) + 1e-12


# ---------------------------------------------------------------------- BA
def test_project_and_residuals_match_oracle(core):
    from BundleAdjustment import bundle_adjustment_residuals, project_points
    p = syn.ba_problem(5, 300, 3, seed=1)
    cams = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    params = np.concatenate([cams.ravel(), p["X0"].ravel()])
    r = bundle_adjustment_residuals(params, 5, 300, p["cam_idx"], p["pt_idx"], p["obs"], K)
    ro = O.ba_residuals(cams, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    assert rel(r, ro) < 1e-9
    x = project_points(K, p["C0"][2], p["R0"][2], p["X0"])
    xo = (K @ (p["R0"][2] @ (p["X0"] - p["C0"][2]).T)).T
    xo = xo[:, :2] / (xo[:, 2:3] + 1e-8)
    assert rel(x, xo) < 1e-9


def _rmse_of(R_set, C_set, Xw, prob, rows=None):
    nc = len(R_set)
    cams = np.concatenate([np.concatenate([O.R_to_rotvec(np.asarray(R_set[i])), -np.asarray(R_set[i]) @ C_set[i]])
                           for i in range(nc)]).reshape(nc, 6)
    r = O.ba_residuals(cams, Xw if rows is None else Xw[rows], prob["cam_idx"], prob["pt_idx"], prob["obs"], K)
    return syn.rmse_from_cost(0.5 * r @ r, len(prob["cam_idx"]))


@pytest.mark.parametrize("name,shape", [("tiny2", (2, 20, 2)), ("tiny", (3, 30, 3)),
                                        ("small", (6, 200, 4)), ("cfg3", (6, 2000, 5))])
def test_perform_bundle_adjustment_matches_converged_reference(core, golden, name, shape, capsys):
    from BundleAdjustment import perform_bundle_adjustment
    b = golden("ba.npz")
    nc, npt, k = shape
    p = syn.ba_problem(nc, npt, k, seed=3)
    R0, C0 = [p["R0"][i] for i in range(nc)], [p["C0"][i] for i in range(nc)]
    Xw = p["X0"].copy()
    R1, C1, X1 = perform_bundle_adjustment(Xw, p["filtered_world_coords"], p["feature_x"], p["feature_y"],
                                           p["flags"], R0, C0, K, nc - 1)
    out = capsys.readouterr().out
    assert f"  Bundle adjustment: {nc} cameras, {npt} points, {len(p['cam_idx'])} observations" in out
    assert "  Bundle adjustment completed. Final cost: " in out
    assert X1 is not Xw and np.array_equal(Xw, p["X0"])  # input untouched, copy returned
    n = len(p["cam_idx"])
    rm = _rmse_of(R1, C1, X1, p)
    rc = syn.rmse_from_cost(float(b[f"{name}_cost_conv"]), n)
    assert abs(rm - rc) <= 1e-4 * rc, (rm, rc)
    if f"{name}_shipped_X" in b:
        rs = _rmse_of(b[f"{name}_shipped_R"], b[f"{name}_shipped_C"], b[f"{name}_shipped_X"], p)
        assert rm <= rs + 1e-9


def test_ba_matches_oracle_midsize(core):
    p = syn.ba_problem(12, 5000, 6, seed=5, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    _, _, ro = O.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=100)
    _, _, rg = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=100)
    n = len(p["cam_idx"])
    assert abs(rg["cost0"] - ro["cost0"]) <= 1e-9 * ro["cost0"]
    ro_r, rg_r = syn.rmse_from_cost(ro["cost"], n), syn.rmse_from_cost(rg["cost"], n)
    assert abs(ro_r - rg_r) <= 1e-4 * ro_r


def test_ba_many_cameras_split_rows(core):
    """356 cameras: the Schur sweep splits camera rows over several specs
    (rows longer than a workgroup's lane budget) and the reduced system is
    2136 x 2136 (134 tile columns); three LM iterations against the C oracle."""
    p = syn.ba_problem(356, 2000, 3, seed=11, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    _, _, ro = O.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=3)
    _, _, rg = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=3)
    assert rg["iterations"] == ro["iterations"] and rg["accepted"] == ro["accepted"]
    assert abs(rg["cost"] - ro["cost"]) <= 1e-7 * ro["cost"], (rg["cost"], ro["cost"])


def test_ba_cfg4_matches_oracle(core):
    """cfg4 (50 cams / 100k pts / 1M obs) against the C Schur-LM restatement
    (at cfg4/5 the build's own CPU Schur-LM, itself pinned to
    the reference's least-squares oracle at cfg3): same iteration and
    accepted counts, |RMSE_gpu - RMSE_oracle| <= 1e-4 RMSE_oracle; plus
    determinism run to run and the reported cost being the cost of the
    returned parameters (reference residual, BundleAdjustment.py:43-110)."""
    p = syn.ba_problem_cfg("cfg4", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    c1, x1, r1 = core.ba_lm(*args, max_iterations=50)
    c2, x2, r2 = core.ba_lm(*args, max_iterations=50)
    _, _, ro = O.ba_lm(*args, max_iterations=50)
    n = len(p["cam_idx"])
    assert (r1["iterations"], r1["accepted"], r1["status"]) == (ro["iterations"], ro["accepted"], ro["status"])
    assert abs(r1["cost0"] - ro["cost0"]) <= 1e-9 * ro["cost0"]
    rg, rr = syn.rmse_from_cost(r1["cost"], n), syn.rmse_from_cost(ro["cost"], n)
    assert abs(rg - rr) <= 1e-4 * rr, (rg, rr)
    assert rg < 0.75  # pixel noise sigma 0.5 per axis
    assert r1["cost"] == r2["cost"] and np.array_equal(x1, x2) and np.array_equal(c1, c2)
    r = core.ba_residuals(c1, x1, p["cam_idx"], p["pt_idx"], p["obs"], K)
    assert abs(0.5 * r @ r - r1["cost"]) <= 1e-8 * r1["cost"]


def test_ba_cfg5_matches_oracle(core):
    """cfg5 (200 cams / 500k pts / ~4M obs, reduced system 1200 x 1200 =
    75 tile columns, rows split across specs) against the C Schur-LM
    restatement: same iteration / accepted counts, RMSE within 1e-4, and the
    reported cost is the cost of the returned parameters."""
    p = syn.ba_problem_cfg("cfg5", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    c1, x1, r1 = core.ba_lm(*args, max_iterations=30)
    _, _, ro = O.ba_lm(*args, max_iterations=30)
    n = len(p["cam_idx"])
    assert (r1["iterations"], r1["accepted"], r1["status"]) == (ro["iterations"], ro["accepted"], ro["status"])
    rg, rr = syn.rmse_from_cost(r1["cost"], n), syn.rmse_from_cost(ro["cost"], n)
    assert abs(rg - rr) <= 1e-4 * rr, (rg, rr)
    assert rg < 0.75
    r = core.ba_residuals(c1, x1, p["cam_idx"], p["pt_idx"], p["obs"], K)
    assert abs(0.5 * r @ r - r1["cost"]) <= 1e-8 * r1["cost"]


def test_perform_bundle_adjustment_coo_equals_dense(core, capsys):
    """The COO store path (no dense n_features x n_images matrices) gives the
    dense path's observations, solve and outputs."""
    from BundleAdjustment import perform_bundle_adjustment, perform_bundle_adjustment_coo
    import sfm_io
    p = syn.ba_problem(6, 400, 4, seed=8, dense=True)
    ff = p["flags"]
    f_idx, i_idx = np.nonzero(ff)
    st = sfm_io.MatchStore(ff.shape[0], ff.shape[1], f_idx.astype(np.int32), i_idx.astype(np.int32),
                           p["feature_x"][f_idx, i_idx], p["feature_y"][f_idx, i_idx])
    st.flag[:] = 1
    a = perform_bundle_adjustment(p["X0"], p["filtered_world_coords"], p["feature_x"], p["feature_y"], ff,
                                  list(p["R0"]), list(p["C0"]), K, 2)
    b = perform_bundle_adjustment_coo(p["X0"], p["filtered_world_coords"], st, list(p["R0"]), list(p["C0"]), K)
    assert np.array_equal(a[2], b[2])
    assert all(np.array_equal(u, v) for u, v in zip(a[0], b[0]))
    out = capsys.readouterr().out
    assert out.count("Bundle adjustment completed") == 2


def test_ba_reused_device_blocks_poisoned(core, monkeypatch, capsys):
    """Problems reuse the device blocks, stream and events of destroyed ones
    (the create/destroy cache): with every reused block filled with 0xFF
    first (SFM_POOL_POISON=1) the solves of a sequence of problems -- sizes
    shrinking, so each one gets blocks that held another problem's data --
    are bitwise those of the first, unpoisoned run, through both entries
    (COO arrays and the dense scan)."""
    from BundleAdjustment import perform_bundle_adjustment
    probs = [syn.ba_problem(12, 5000, 6, seed=5, dense=True), syn.ba_problem(10, 3000, 5, seed=6, dense=True),
             syn.ba_problem(8, 2000, 4, seed=7, dense=True)]

    def run():
        out = []
        for p in probs:
            cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
            c, x, rep = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
            d = perform_bundle_adjustment(p["X0"], p["filtered_world_coords"], p["feature_x"], p["feature_y"],
                                          p["flags"], list(p["R0"]), list(p["C0"]), K, 0)
            out.append((c, x, rep["cost"], d[2], np.array(d[0])))
        return out

    clean = run()
    monkeypatch.setenv("SFM_POOL_POISON", "1")
    poisoned = run()
    for a, b in zip(clean, poisoned):
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
    assert capsys.readouterr().out.count("Bundle adjustment completed") == 2 * len(probs)


def test_ba_concurrent_calls_equal_sequential(core):
    """sfm_ba_lm from several host threads at once (ctypes drops the GIL):
    the calls contend for the pinned upload stage, so some take the busy
    path (the COO and x0 from pageable memory, no second stream) while one
    holds the stage (indices first, coordinates and points on the stage's
    second stream).  Every concurrent result is bitwise the sequential one."""
    import threading
    probs = [syn.ba_problem(12, 20000, 6, seed=s, dense=False) for s in (11, 12, 13, 14)]
    args = [(np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])]), p["X0"], p["cam_idx"],
             p["pt_idx"], p["obs"], K) for p in probs]
    seq = [core.ba_lm(*a, max_iterations=15) for a in args]
    for _ in range(2):
        out, errs = [None] * len(args), []

        def run(i):
            try:
                out[i] = core.ba_lm(*args[i], max_iterations=15)
            except Exception as e:  # reported below
                errs.append(repr(e))

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(args))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs, errs
        for (c0, x0, r0), (c1, x1, r1) in zip(seq, out):
            assert r1["iterations"] == r0["iterations"] and r1["cost"] == r0["cost"]
            assert np.array_equal(c1, c0) and np.array_equal(x1, x0)


def test_ba_failure_contract(core, capsys):
    from BundleAdjustment import perform_bundle_adjustment
    p = syn.ba_problem(3, 30, 2, seed=2)  # 2*60 residuals < 18 + 90 params? no: 120 >= 108
    R0, C0 = [p["R0"][i] for i in range(3)], [p["C0"][i] for i in range(3)]
    # too few observations -> scipy's m < n error, inputs returned as the same objects
    flags = p["flags"].copy()
    flags[:, 2] = 0
    Xw = p["X0"].copy()
    R1, C1, X1 = perform_bundle_adjustment(Xw, p["filtered_world_coords"], p["feature_x"], p["feature_y"],
                                           flags, R0, C0, K, 2)
    assert R1 is R0 and C1 is C0 and X1 is Xw
    assert "Bundle adjustment failed: Method 'lm' doesn't work" in capsys.readouterr().out
    # no valid points -> inputs, nothing printed
    R1, C1, X1 = perform_bundle_adjustment(Xw, 0 * p["filtered_world_coords"], p["feature_x"], p["feature_y"],
                                           p["flags"], R0, C0, K, 2)
    assert X1 is Xw and capsys.readouterr().out == ""
    # a non-finite residual at x0 (scipy least_squares.py:843-845): the
    # device's initial cost ends the solve (status 6) and the drop-in fails
    Xn = p["X0"].copy()
    Xn[3, 1] = np.nan
    R1, C1, X1 = perform_bundle_adjustment(Xn, p["filtered_world_coords"], p["feature_x"], p["feature_y"],
                                           p["flags"], R0, C0, K, 2)
    assert R1 is R0 and C1 is C0 and X1 is Xn
    assert "Bundle adjustment failed: Residuals are not finite in the initial point." in capsys.readouterr().out
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    _, _, rep = core.ba_lm(cams0, Xn, p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=20)
    assert rep["status"] == 6 and rep["iterations"] == 0 and not np.isfinite(rep["cost0"])
    # finite residuals whose squared sum overflows (|r| ~ 1e163 px): a known
    # divergence, DESIGN §3.  scipy checks the residual vector (finite) and
    # MINPACK's overflow-safe enorm runs the solve with cost = inf; the device
    # tests the summed cost and ends the solve as for a non-finite residual
    cams = np.zeros((3, 6))
    cams[:, 3] = [0.1, -0.2, 0.3]
    rng = np.random.default_rng(5)
    X = np.column_stack([rng.uniform(-1, 1, (20, 2)), rng.uniform(4, 8, 20)])
    X[7] = [1e160, 0.0, 1.0]  # camera frame (1e160 + tx, 0, 1): u = fx * 1e160
    ci, pi = np.tile(np.arange(3), 20).astype(np.int32), np.repeat(np.arange(20), 3).astype(np.int32)  # point-major
    obs = rng.uniform(0, 500, (60, 2))
    _, _, rep = core.ba_lm(cams, X, ci, pi, obs, K, max_iterations=20)
    assert rep["status"] == 6 and rep["iterations"] == 0 and np.isinf(rep["cost0"])


def _spd(n, seed, cond=1e4):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = np.logspace(0, np.log10(cond), n)
    S = (Q * ev) @ Q.T
    return 0.5 * (S + S.T), rng.standard_normal(n)


@pytest.mark.parametrize("solver", ["gj", "gjseg", "chol"])
@pytest.mark.parametrize("n", [1, 6, 16, 17, 48, 150, 300, 304, 600, 1200, 1800, 2100])
def test_reduced_solve(core, monkeypatch, n, solver):
    """The reduced-camera solvers against LAPACK on SPD systems with condition
    number 1e4: the row-distributed persistent block Gauss-Jordan solve
    (default; gjr_solve.hpp, up to 128 tile rows -- n = 2100 falls back to
    the tiled Cholesky), the column-block segment Gauss-Jordan solve
    (SFM_SOLVE=gjseg, gj_solve.hpp: the live fallback when the row layout
    declines) and the tiled Cholesky (SFM_SOLVE=chol: k_chol_col launches,
    forward substitution folded in, back substitution).  Relative error
    <= 1e-11 (all backward stable; kappa * eps ~ 2e-12); deterministic."""
    monkeypatch.setenv("SFM_SOLVE", solver)
    S, b = _spd(n, seed=n)
    x_ref = np.linalg.solve(S, b)
    x = core.reduced_solve(S, b)
    assert np.abs(x - x_ref).max() <= 1e-11 * np.abs(x_ref).max(), np.abs(x - x_ref).max()
    assert np.array_equal(x, core.reduced_solve(S, b))


@pytest.mark.parametrize("solver", ["gj", "gjseg", "chol"])
@pytest.mark.parametrize("n", [40, 300, 1200])
def test_reduced_solve_not_spd(core, monkeypatch, n, solver):
    """A non-positive pivot is reported by either solver."""
    monkeypatch.setenv("SFM_SOLVE", solver)
    S, b = _spd(n, seed=1)
    S[7, 7] = -1.0
    with pytest.raises(RuntimeError, match="positive definite"):
        core.reduced_solve(S, b)


@pytest.mark.parametrize("shape", ["cfg4", "cfg5"])
def test_ba_gj_solve_matches_cholesky(core, monkeypatch, shape):
    """The whole LM solve with the persistent Gauss-Jordan reduced solve
    (default) and with the tiled Cholesky (SFM_SOLVE=chol): the same
    accept/reject sequence and cost to 1e-9 relative (the two solvers round
    differently, so the steps agree to ~1e-12, not bitwise)."""
    p = syn.ba_problem_cfg(shape, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    out = {}
    for solver in ("gj", "chol"):
        monkeypatch.setenv("SFM_SOLVE", solver)
        out[solver] = core.ba_lm(*args, max_iterations=30)
    (cg, xg, rg), (cc, xc, rc) = out["gj"], out["chol"]
    assert (rg["iterations"], rg["accepted"], rg["status"]) == (rc["iterations"], rc["accepted"], rc["status"])
    assert abs(rg["cost"] - rc["cost"]) <= 1e-9 * rc["cost"]
    assert np.abs(cg - cc).max() < 1e-8 and np.abs(xg - xc).max() < 1e-6


def test_ba_sweep_pinhole_matches_general_k(core, monkeypatch):
    """The Schur sweep's pinhole-K pair math (the five zeros of K dropped,
    default for the reference's calibration) against the general-K path
    (SFM_SWEEP_PINHOLE=0) on cfg4: the same accept/reject sequence, cost
    within 1e-9 relative (the Hessian's products round differently)."""
    p = syn.ba_problem_cfg("cfg4", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    c1, x1, r1 = core.ba_lm(*args, max_iterations=30)
    monkeypatch.setenv("SFM_SWEEP_PINHOLE", "0")
    c0, x0, r0 = core.ba_lm(*args, max_iterations=30)
    assert (r1["iterations"], r1["accepted"], r1["status"]) == (r0["iterations"], r0["accepted"], r0["status"])
    assert abs(r1["cost"] - r0["cost"]) <= 1e-9 * r0["cost"]


@pytest.mark.parametrize("shape", ["cfg4", "cfg5", "many"])
def test_ba_device_plan_equals_host_plan(core, monkeypatch, shape):
    """The Schur sweep plan built on the device at create (the chunk
    statistics, the per-chunk pair counts and the (chunk, spec) slot / pair
    lists from the uploaded COO) is the host planner's plan (SFM_PLAN_HOST=1)
    byte for byte: the same digest over every plan array, the lists read back
    from the device in both cases.  "many": 356 cameras, long rows split over
    several specs (its block counts exceed the LDS histograms: the global
    atomic kernels).  The device's global-atomic forms of the block counts,
    per-chunk counts and chunk statistics (round 5's LDS-histogram kernels
    off) give the same plan too."""
    p = syn.ba_problem_cfg(shape, dense=False) if shape != "many" else syn.ba_problem(356, 2000, 3, seed=11,
                                                                                     dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    monkeypatch.setenv("SFM_PLAN_DIGEST", "1")
    dig = {}
    for host, glob in (("0", "0"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("SFM_PLAN_HOST", host)
        for e in ("SFM_CSR_CNT_GLOBAL", "SFM_PLAN_COUNTS_GLOBAL"):
            monkeypatch.setenv(e, glob)
        if glob == "1":
            monkeypatch.setenv("SFM_PLAN_CHUNK_SPLIT", "1")
        else:
            monkeypatch.delenv("SFM_PLAN_CHUNK_SPLIT", raising=False)
        prob = core.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
        dig[host, glob] = prob.plan_digest()
        prob.close()
    assert dig["0", "0"] != 0 and dig["0", "0"] == dig["1", "0"] == dig["0", "1"], dig


def test_ba_sweep_split_and_gjr_fold_paths(core, monkeypatch):
    """cfg5, where the Schur sweep's last dispatch round is cut into chunk
    sub-ranges (SweepSplit, split_S = 8 by default): the split plan against
    the unsplit one (SFM_SWEEP_SPLIT=0: the same blocks summed in another
    order, so the LM agrees to rounding), and k_schur_finish folded into the
    row solve's prologue (SFM_GJR_FOLD=1: the slabs read in the finish's
    order, camera U / g from the camera-block partials) against the finish
    launch: the same sums in the same order, so bitwise the same solve.
    The split needs 8 ranges (one a XCD); cfg5 plans 2 by default since
    round 5, so the test asks for 8, and the default plan joins the
    comparison."""
    p = syn.ba_problem_cfg("cfg5", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    out = {}
    out["default", "0"] = core.ba_lm(*args, max_iterations=12)
    monkeypatch.setenv("SFM_SWEEP_RANGES", "8")
    for split, fold in (("8", "0"), ("0", "0"), ("8", "1"), ("0", "1")):
        monkeypatch.setenv("SFM_SWEEP_SPLIT", split)
        monkeypatch.setenv("SFM_GJR_FOLD", fold)
        out[split, fold] = core.ba_lm(*args, max_iterations=12)
    c8, x8, r8 = out["8", "0"]
    for key, (c, x, r) in out.items():
        assert (r["iterations"], r["accepted"], r["status"]) == (r8["iterations"], r8["accepted"], r8["status"]), key
        assert abs(r["cost"] - r8["cost"]) <= 1e-9 * r8["cost"], key
        assert np.abs(c - c8).max() < 1e-8 and np.abs(x - x8).max() < 1e-6, key
    for split in ("8", "0"):  # the fold is the finish's arithmetic
        (ca, xa, ra), (cb, xb, rb) = out[split, "0"], out[split, "1"]
        assert ra["cost"] == rb["cost"] and np.array_equal(ca, cb) and np.array_equal(xa, xb), split


@pytest.mark.parametrize("shape,ranks", [("cfg4", 4), ("cfg5", 8)])
def test_ba_multi_rank_baseline_sizes(core, shape, ranks):
    """The point-sharded LM at BASELINE's sizes (cfg4 on 4, cfg5 on 8
    in-process ranks sharing the one GPU: partial reduced camera systems
    all-reduced every iteration, every rank running the replicated
    persistent solve) against the single-rank solve: the same iteration and
    accepted counts, cost within 1e-9 relative."""
    p = syn.ba_problem_cfg(shape, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    c1, x1, r1 = core.ba_lm(*args, max_iterations=30)
    cN, xN, rN = core.ba_lm_multi(*args, [0] * ranks, max_iterations=30)
    assert rN["n_ranks"] == ranks
    assert (rN["iterations"], rN["accepted"], rN["status"]) == (r1["iterations"], r1["accepted"], r1["status"])
    assert abs(rN["cost"] - r1["cost"]) <= 1e-9 * r1["cost"]
    assert np.abs(cN - c1).max() < 1e-8 and np.abs(xN - x1).max() < 1e-6


@pytest.mark.parametrize("ranks", [2, 3])
def test_ba_multi_rank_matches_single_rank(core, ranks):
    """The point-sharded LM (one partial reduced camera system per rank,
    summed every iteration) on several ranks sharing the one GPU gives the
    single-rank result: same accept/reject sequence, RMSE equal to 1e-9."""
    p = syn.ba_problem(20, 20000, 6, seed=6, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    c1, x1, r1 = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=40)
    cN, xN, rN = core.ba_lm_multi(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, [0] * ranks,
                                  max_iterations=40)
    assert rN["n_ranks"] == ranks
    assert rN["iterations"] == r1["iterations"] and rN["accepted"] == r1["accepted"]
    assert abs(rN["cost"] - r1["cost"]) <= 1e-9 * r1["cost"]
    assert np.abs(xN - x1).max() < 1e-6 and np.abs(cN - c1).max() < 1e-8


def test_ba_through_rccl_communicator(core):
    """The one-process-per-GPU transport: a real RCCL communicator (one rank
    here) carries the per-iteration all-reduces; same result as no comm."""
    p = syn.ba_problem(8, 3000, 4, seed=8, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    uid = core.Comm.unique_id()
    comm = core.Comm(uid, 1, 0)
    try:
        prob = core.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, comm=comm)
        rep = prob.solve(max_iterations=30)
        c1, x1 = prob.download()
        prob.close()
    finally:
        comm.close()
    c0, x0, rep0 = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K, max_iterations=30)
    assert rep["n_ranks"] == 1 and rep["iterations"] == rep0["iterations"]
    assert rep["cost"] == rep0["cost"] and np.array_equal(x1, x0)


def test_bench_multi_rank_entry_runs_under_torchrun(tmp_path):
    """bench.py's N>1 code path (gloo control plane + RCCL data plane) with
    WORLD_SIZE=1 under torch.distributed.run, small workload."""
    import subprocess
    import sys
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=29517", os.path.join(repo, "bench.py"), "--gpus", "1",
           "--steps", "3", "--warmup", "1", "--workload", "cfg3", "--no-cpu-baseline", "--ransac-hyps", "512",
           "--force-comm"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 1 and d["value"] > 0


@pytest.mark.parametrize("gtol", [1e9, 1e3, 1.0, 1e-2])
def test_ba_gradient_tolerance_stop(core, gtol):
    """gradient_tolerance: the stop after a linearisation when max |J^T r| <
    gtol (status 2, the iteration not counted), as orc_ba_lm does; single
    rank and two in-process ranks (the count and g_c are all-reduced)."""
    p = syn.ba_problem(8, 600, 4, seed=5, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    _, _, ro = O.ba_lm(*args, max_iterations=50, gtol=gtol, ftol=1e-10)
    assert ro["status"] == 2
    c1, x1, rg = core.ba_lm(*args, max_iterations=50, gradient_tolerance=gtol)
    _, _, rm = core.ba_lm_multi(*args, devices=[0, 0], max_iterations=50, gradient_tolerance=gtol)
    for r in (rg, rm):
        assert r["status"] == 2, r
        assert (r["iterations"], r["accepted"]) == (ro["iterations"], ro["accepted"])
        assert abs(r["cost"] - ro["cost"]) <= 1e-9 * ro["cost"]
    if ro["iterations"] == 0:
        assert np.array_equal(x1, p["X0"]) and rg["cost"] == rg["cost0"]
    with pytest.raises(Exception):
        core.ba_lm(*args, max_iterations=5, gradient_tolerance=-1.0)


def test_ransac_combine_through_rccl_communicator(core):
    """sfm_ransac_combine's RCCL path (all-reduce(max, u64) of the key, then
    the winner's model as a sum) with a one-rank communicator: the shard's
    key and model come back unchanged, repeatedly (cached scratch)."""
    import sfm_dist
    x1, x2, _, _ = syn.two_view(n=2000, seed=9)
    random.seed(5)
    key, F, _ = core.ransac_f8_range(x1, x2, 700, 0, 700, 0.06)
    assert key != 0
    comm = core.Comm(core.Comm.unique_id(), 1, 0)
    try:
        for _ in range(3):
            k2, F2 = core.ransac_combine(comm, key, F)
            assert k2 == key and np.array_equal(F2, F)
        k0, _ = core.ransac_combine(comm, 0, np.zeros(9))
        assert k0 == 0
    finally:
        comm.close()
    random.seed(5)
    b, Fb, mask, _, _ = core.ransac_f8_pyrandom(x1, x2, 700, 0.06)
    assert sfm_dist.key_iter(key)[1] == b and np.array_equal(F, Fb)
    assert np.array_equal(core.ransac_mask(x1, x2, F, 0.06), mask)


def test_ba_camera_blocks_fused_equal_standalone(core, monkeypatch):
    """The camera blocks of the normal equations computed by extra workgroups
    of the Schur sweep (default) and by the standalone k_camera_lin
    (SFM_CAMLIN_FUSED=0): the same LM trajectory (counts, status) and final
    cost within 1e-10 (the two cut each camera's observations into different
    items, so the sums differ in order only)."""
    p = syn.ba_problem_cfg("cfg3", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    reps = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("SFM_CAMLIN_FUSED", fused)
        _, _, reps[fused] = core.ba_lm(*args, max_iterations=30)
    a, b = reps["1"], reps["0"]
    assert (a["iterations"], a["accepted"], a["status"]) == (b["iterations"], b["accepted"], b["status"])
    assert abs(a["cost"] - b["cost"]) <= 1e-10 * b["cost"]


@pytest.mark.parametrize("shape", ["cfg3", "50x6000"])
def test_ba_solve_variants_bitwise_equal(core, monkeypatch, shape):
    """The tiled Cholesky reduced solve (SFM_SOLVE=chol): its DPP tile factor (default) and the readlane chain
    (SFM_CHOL_DPP=0), and the Schur finish folded into the solve's first
    launch at one rank (default) or run as its own launch
    (SFM_FINISH_FUSED=0): the same operations in the same order, so the
    whole LM solve -- counts, status, cost, cameras and points -- is bitwise
    the same in all four combinations.  50x6000: 19 tile columns, as cfg4."""
    if shape == "cfg3":
        p = syn.ba_problem_cfg("cfg3", dense=False)
    else:
        p = syn.ba_problem(50, 6000, 8, seed=5)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    out = {}
    monkeypatch.setenv("SFM_SOLVE", "chol")  # the variants are the tiled Cholesky's
    for dpp in ("1", "0"):
        for fin in ("1", "0"):
            monkeypatch.setenv("SFM_CHOL_DPP", dpp)
            monkeypatch.setenv("SFM_FINISH_FUSED", fin)
            out[dpp + fin] = core.ba_lm(*args, max_iterations=12, fixed_iterations=True)
    c0, x0, r0 = out["11"]
    assert r0["accepted"] > 0
    for key, (c, x, r) in out.items():
        assert (r["iterations"], r["accepted"], r["status"], r["cost"]) == \
            (r0["iterations"], r0["accepted"], r0["status"], r0["cost"]), key
        assert np.array_equal(c, c0) and np.array_equal(x, x0), key


def test_ba_timing_and_lm_state_polling(core):
    """Per-phase kernel times are recorded only with sfm_ba_set_timing on,
    and turning them on does not change the solve; a solve that converges
    early stops there (the host reads the LM state from the pinned ring, at
    most two gated-off iterations follow) and a repeated solve is bitwise
    the same."""
    p = syn.ba_problem_cfg("cfg3", dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    prob = core.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    try:
        r0 = prob.solve(max_iterations=200)
        assert r0["status"] in (1, 3) and r0["iterations"] < 200
        assert all(v == 0.0 for v in prob.kernel_times().values())
        c0, x0 = prob.download()
        prob.reset()
        prob.set_timing(True)
        r1 = prob.solve(max_iterations=200)
        kt = prob.kernel_times()
        assert kt["schur_blocks"] > 0 and kt["cholesky"] > 0
        c1, x1 = prob.download()
        assert (r1["iterations"], r1["accepted"], r1["cost"]) == (r0["iterations"], r0["accepted"], r0["cost"])
        assert np.array_equal(c0, c1) and np.array_equal(x0, x1)
        prob.set_timing(False)
        for it in (1, 2, 3):  # stops exactly at max_iterations when it has not converged
            prob.reset()
            assert prob.solve(max_iterations=it, fixed_iterations=True)["iterations"] == it
    finally:
        prob.close()


def test_call_timing_switch(core):
    """The drop-in RANSAC call records device timings only with
    sfm_set_call_timing on; the host sampling time is always reported, and
    the result does not depend on the switch."""
    x1, x2, _, _ = syn.two_view(n=1500, seed=3)
    out = []
    for on in (False, True, False):
        core.set_call_timing(on)
        random.seed(11)
        out.append(core.ransac_f8_pyrandom(x1, x2, 900, 0.06, want_counts=True))
        t = core.last_timings()
        assert (t[1] > 0) == on and t[6] > 0
    b0, M0, m0, c0 = out[0][:4]
    for b, M, m, c in (o[:4] for o in out[1:]):
        assert b == b0 and np.array_equal(c, c0) and np.array_equal(m, m0) and np.array_equal(M, M0)


def _thresholds_at(d, n=24):
    """thresholds sitting exactly on (and one ulp either side of) n of the
    given distances: every one of those pairs lies in the fast test's band"""
    d = d[np.isfinite(d) & (d > 1e-6) & (d < 1e6)]
    pick = np.sort(d)[np.linspace(0, len(d) - 1, n).astype(int)]
    return np.concatenate([pick, np.nextafter(pick, np.inf), np.nextafter(pick, -np.inf)])


def test_ransac_fast_tests_exact_at_threshold(core):
    """The score kernels' fast tests (the two-stage epipolar test with its
    wave-level outlier skip, the homography transfer-error test) against the
    ORACLE's distances (the reference expressions GetInliersRANSAC.py:67-78
    and GetHomographyInliers.py:136-142, equal to numpy's bit for bit:
    test_oracle.py), with thresholds placed exactly on (and one ulp around)
    those distances: the count of one hypothesis (fast path + exact tail),
    the winner's mask (select kernel) and the standalone mask all equal the
    oracle's strict test err < thr."""
    x1, x2, _, _ = syn.two_view(n=3000, seed=11)
    random.seed(4)
    sample = np.array([random.sample(range(len(x1)), 8)], dtype=np.int32)
    b, F, _, _ = core.ransac_f8(x1, x2, sample, 1e3, want_counts=True)
    assert b == 0
    err = O.epi_err(x1, x2, F)
    for thr in _thresholds_at(err):
        ref = err < thr
        assert np.array_equal(ref, O.ransac_mask(x1, x2, F, float(thr)))
        b, Fb, mask, counts = core.ransac_f8(x1, x2, sample, float(thr), want_counts=True)
        assert counts[0] == ref.sum(), thr
        assert np.array_equal(core.ransac_mask(x1, x2, F, float(thr), model=8), ref), thr
        if counts[0] > 0:
            assert b == 0 and np.array_equal(Fb, F) and np.array_equal(mask, ref), thr
    # homography: one in-call hypothesis from a fixed stream, thresholds on its transfer errors
    random.seed(9)
    b, Hm, _, _, _ = core.ransac_h4_pyrandom(x1, x2, 1, 1e6)
    assert b == 0
    err = O.hom_err(x1, x2, Hm)
    for thr in _thresholds_at(err):
        ref = err < thr
        random.seed(9)
        b, Hb, mask, counts, _ = core.ransac_h4_pyrandom(x1, x2, 1, float(thr), want_counts=True)
        assert counts[0] == ref.sum(), thr
        assert np.array_equal(core.ransac_mask(x1, x2, Hm, float(thr), model=4), ref), thr
        if counts[0] > 0:
            assert np.array_equal(mask, ref), thr


@pytest.mark.parametrize("scale", [1e-3, 1.0, 1e3, 1e5, 3e7])
def test_ransac_float_prefilter_never_changes_a_count(core, monkeypatch, scale):
    """The score's float prefilter (sfm_geom.hpp epi_pre_setup / epi_pre_test:
    packed FP32, proving outliers with a rigorous error bound) leaves every
    per-hypothesis count equal to the reference expression's count with that
    hypothesis' F (O.epi_err, bit-exact to numpy) and to the counts without
    the prefilter (SFM_SCORE_PRE=0): coordinates from 1e-3 to 3e7 (above
    2^24 the prefilter switches itself off), thresholds placed on the first
    hypothesis' distances and one ulp around them, a NaN correspondence (its
    tile's bound is inf) and both entries (given table, in-call draws)."""
    x1, x2, _, _ = syn.two_view(n=2500, seed=13)
    x1, x2 = x1 * scale, x2 * scale
    x1[1700] = np.nan
    rng = np.random.default_rng(5)
    H = 48
    samples = np.stack([rng.choice(1600, 8, replace=False) for _ in range(H)]).astype(np.int32)
    # each hypothesis' F as the score sees it: the winner of a one-row table
    Fs = [core.ransac_f8(x1, x2, samples[h:h + 1], 1e300)[1] for h in range(H)]
    errs = [O.epi_err(x1, x2, F) for F in Fs]
    d = np.sort(errs[0][np.isfinite(errs[0]) & (errs[0] > 0)])
    pick = d[(np.array([0.005, 0.05, 0.3]) * (len(d) - 1)).astype(int)]
    for thr in list(pick) + list(np.nextafter(pick, np.inf)) + list(np.nextafter(pick, -np.inf)) + [0.5 * scale]:
        ref = np.array([(e < thr).sum() for e in errs], dtype=np.int32)
        monkeypatch.delenv("SFM_SCORE_PRE", raising=False)
        got = core.ransac_f8(x1, x2, samples, float(thr), want_counts=True)[3]
        random.seed(21)
        pyr = core.ransac_f8_pyrandom(x1, x2, 40, float(thr), want_counts=True)[3]
        monkeypatch.setenv("SFM_SCORE_PRE", "0")
        off = core.ransac_f8(x1, x2, samples, float(thr), want_counts=True)[3]
        random.seed(21)
        pyr_off = core.ransac_f8_pyrandom(x1, x2, 40, float(thr), want_counts=True)[3]
        assert np.array_equal(got, ref), thr
        assert np.array_equal(off, ref), thr
        assert np.array_equal(pyr, pyr_off), thr


def test_ransac_launcher_thread_equals_one_thread(core, monkeypatch):
    """The in-call pipeline's two host threads (the caller draws, a pool
    worker enqueues each chunk's launches as its rows are published) against
    the one-thread order (SFM_RANSAC_LAUNCHER=0): the same counts, winner,
    F and mask, and the global random stream left in the same state; F and
    H models."""
    x1, x2, _, _ = syn.two_view(n=5000, seed=0)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SFM_RANSAC_LAUNCHER", mode)
        random.seed(7)
        f = core.ransac_f8_pyrandom(x1, x2, 16384, 0.06, want_counts=True)
        st_f = random.getstate()
        random.seed(7)
        h = core.ransac_h4_pyrandom(x1, x2, 4096, 30.0, want_counts=True)
        out[mode] = (f, st_f, h, random.getstate())
    (f1, s1, h1, t1), (f0, s0, h0, t0) = out["1"], out["0"]
    for a, b in ((f1, f0), (h1, h0)):
        assert a[0] == b[0]
        for x, y in zip(a[1:4], b[1:4]):
            assert np.array_equal(np.asarray(x), np.asarray(y))
    assert s1 == s0 and t1 == t0


def test_ransac_score_queue_overflow(core, monkeypatch):
    """k_epi_score's survivor queue past its capacity: a threshold far above
    every distance (but below the prefilter's own cutoff) leaves every pair
    a candidate, so each workgroup queues 4096 of its ~20,000 (4 hypotheses
    x 5,000 pairs) and tests the rest in place.  Counts equal the FP64 path's
    (SFM_SCORE_PRE=0) and, for the first hypotheses, the reference
    expression's (O.epi_err with the hypothesis' own F); a second case puts
    the pairs over several ranges (atomically summed counts)."""
    x1, x2, _, _ = syn.two_view(n=5000, seed=3)
    random.seed(3)
    samples = core.sample_table(5000, 8, 2048)
    for thr in (1e5, 40.0):
        monkeypatch.delenv("SFM_SCORE_PRE", raising=False)
        got = core.ransac_f8(x1, x2, samples, thr, want_counts=True)[3]
        monkeypatch.setenv("SFM_SCORE_PRE", "0")
        off = core.ransac_f8(x1, x2, samples, thr, want_counts=True)[3]
        assert np.array_equal(got, off), thr
        for h in range(4):
            F = core.ransac_f8(x1, x2, samples[h:h + 1], 1e300)[1]
            assert got[h] == (O.epi_err(x1, x2, F) < thr).sum(), (thr, h)
    monkeypatch.delenv("SFM_SCORE_PRE", raising=False)
    xa, xb, _, _ = syn.two_view(n=20011, seed=4)  # 157 passes, the last partial
    few = samples[:24] % 20011
    got = core.ransac_f8(xa, xb, few, 1e5, want_counts=True)[3]
    monkeypatch.setenv("SFM_SCORE_PRE", "0")
    assert np.array_equal(got, core.ransac_f8(xa, xb, few, 1e5, want_counts=True)[3])


def test_pnp_fast_test_exact_at_threshold(core):
    """The PnP score kernel's fast reprojection test (v_rcp_f64 + Newton, a
    widened band, the exact tail inside it; pnp.hip pnp_fast) against the
    oracle's reprojection errors (PnPRANSAC.py:60-68, numpy's bit for bit),
    thresholds exactly on (and one ulp around) them: the hypothesis count
    equals the oracle's strict test on the winning pose."""
    X, x, Ct, Rt = _pnp_scene(4000, 21, outlier_frac=0.2)
    random.seed(21)
    samples = core.sample_table(len(X), 4, 256)
    _, _, _, _, counts, branches = core.pnp_ransac(X, x, K, samples, 8.0, want_counts=True)
    # hypotheses off the det(R) < 0 branch (parity unpinned by construction,
    # DESIGN §3), the best-supported first
    hs = [h for h in np.argsort(-counts, kind="stable") if branches[h] == 0][:3]
    assert hs
    checked = 0
    for h in hs:
        one = samples[h:h + 1]
        b0, _, C, R, _, _ = core.pnp_ransac(X, x, K, one, 1e4, want_counts=True)
        assert b0 == 0  # every point an inlier: the hypothesis's pose comes back
        err = O.pnp_err(X, x, K, C, R)
        for thr in _thresholds_at(err[err < 50.0]):
            b1, c1, C1, R1, cnt, br = core.pnp_ransac(X, x, K, one, float(thr), want_counts=True)
            assert br[0] == 0
            assert cnt[0] == (err < thr).sum(), thr
            if b1 == 0:  # a winner (>= 4 inliers): its pose is the hypothesis's
                assert np.array_equal(C1, C) and np.array_equal(R1, R)
            checked += 1
    assert checked > 0


@pytest.mark.parametrize("shape", ["cfg3", "300x6000"])
def test_ba_camera_lds_paths_match_global(core, monkeypatch, shape):
    """k_backsub_trial and k_linearize with the cameras staged in LDS
    (default) against the per-observation camera gathers
    (SFM_BACKSUB_CAM_LDS=0, SFM_LINEARIZE_CAM_LDS=0): the per-point values
    are the same bits, only the block partials of the costs are summed over
    a different grid, so the LM trajectory (counts, status) is the same and
    the cost, cameras and points agree to rounding.  300x6000: 300 cameras
    are 72 KB of back-substitution cameras, past the 64-KB LDS stage, so
    that kernel falls back to the gathers while k_linearize (29 KB) stages."""
    if shape == "cfg3":
        p = syn.ba_problem_cfg("cfg3", dense=False)
    else:
        p = syn.ba_problem(300, 6000, 8, seed=7)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    args = (cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], K)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SFM_BACKSUB_CAM_LDS", v)
        monkeypatch.setenv("SFM_LINEARIZE_CAM_LDS", v)
        out[v] = core.ba_lm(*args, max_iterations=20)
    (ca, Xa, a), (cb, Xb, b) = out["1"], out["0"]
    assert (a["iterations"], a["accepted"], a["status"]) == (b["iterations"], b["accepted"], b["status"])
    assert abs(a["cost"] - b["cost"]) <= 1e-10 * b["cost"]
    assert np.allclose(ca, cb, rtol=0, atol=1e-8) and np.allclose(Xa, Xb, rtol=0, atol=1e-8)
