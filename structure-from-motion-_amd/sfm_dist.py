"""Multi-GPU partitioning of the hot path.

* BA: points -- with all of their observations -- are split into contiguous
  ranges, one per rank; every rank holds every camera.  Each observation
  lives on exactly one rank, so the per-rank partial reduced camera systems
  simply add (one RCCL all-reduce per LM iteration, csrc/ba.hip).
* RANSAC: hypotheses are split into contiguous ranges; the global winner is
  (max count, then min iteration), i.e. the reference's strict '>' rule
  applied across ranks, found as the max of a packed 64-bit key.  The sample
  table is drawn whole, in the reference's order, on every rank (the global
  random stream ends where the unsharded call leaves it).
* LinearTriangulation: contiguous point ranges, no collective; the ranges
  are gathered in rank order (triangulate_sharded).
* Image pairs: the driver's pair loop (Wrapper_dev.py:67-123) spread over
  ranks (pair_loop_spread).  Every rank replays the global random stream
  through the whole loop -- each pair's homography RANSAC, then the draw of
  its F sample table -- because the F table's N is the homography inlier
  count and every draw shifts the stream for the next pair; the F-RANSACs,
  scored from the drawn tables, are split round-robin over the ranks.
"""
import numpy as np


def point_range(n_pts, world, rank):
    lo = (n_pts * rank) // world
    hi = (n_pts * (rank + 1)) // world
    return lo, hi


def shard_ba(cam_idx, pt_idx, obs, X0, world, rank):
    """Observations must be point-major.  Returns the rank's (cam_idx,
    pt_idx rebased to 0, obs, X0 rows, (lo, hi))."""
    pt_idx = np.asarray(pt_idx)
    lo, hi = point_range(len(X0), world, rank)
    o0 = int(np.searchsorted(pt_idx, lo, side="left"))
    o1 = int(np.searchsorted(pt_idx, hi, side="left"))
    return (np.ascontiguousarray(cam_idx[o0:o1]), np.ascontiguousarray(pt_idx[o0:o1] - lo),
            np.ascontiguousarray(obs[o0:o1]), np.ascontiguousarray(X0[lo:hi]), (lo, hi))


def hypothesis_range(H, world, rank):
    return (H * rank) // world, (H * (rank + 1)) // world


def shard_key(count, it):
    """The reference keeps the max count and, among equal counts, the
    earliest iteration (strict '>' update, GetInliersRANSAC.py:85-88): the
    max over ranks of (count << 32) | (0xFFFFFFFF - iteration).  0 = no
    hypothesis with an inlier."""
    return (int(count) << 32) | (0xFFFFFFFF - int(it)) if count > 0 and it >= 0 else 0


def key_iter(key):
    """(count, iteration) of a shard key, (0, -1) for key 0."""
    key = int(key)
    if key == 0:
        return 0, -1
    return key >> 32, 0xFFFFFFFF - (key & 0xFFFFFFFF)


def combine_ransac(per_rank):
    """per_rank: list of (best_count, best_global_iter or -1) -> (count, iter)."""
    return key_iter(max(shard_key(c, i) for c, i in per_rank) if per_rank else 0)


def combine_keys_torch(key, model, group=None):
    """The shard combine over a torch.distributed group (gloo on the CPU
    tests): all-reduce(max) of the keys, then the winner's model as a sum in
    which only the rank holding the max key contributes.  Keys fit int64
    (counts < 2^31)."""
    import torch
    import torch.distributed as dist
    k = torch.tensor([int(key)], dtype=torch.int64)
    dist.all_reduce(k, op=dist.ReduceOp.MAX, group=group)
    g = int(k.item())
    mine = np.asarray(model, dtype=np.float64).reshape(9) if (g != 0 and int(key) == g) else np.zeros(9)
    m = torch.tensor(mine, dtype=torch.float64)
    dist.all_reduce(m, op=dist.ReduceOp.SUM, group=group)
    return g, m.numpy().reshape(3, 3)


def ransac_sharded(n_corr, H, rank, world, shard_fn, combine_fn, mask_fn):
    """Hypothesis-sharded RANSAC: this rank fits and scores
    hypotheses [h0, h1) -- shard_fn(h0, h1) -> (key, model) --, the ranks
    combine keys (combine_fn(key, model) -> (key, model)), and the winner's
    model gives the mask (mask_fn(model)).  Returns the unsharded call's
    (best iteration or -1, model or None, mask)."""
    h0, h1 = hypothesis_range(H, world, rank)
    key, model = shard_fn(h0, h1)
    key, model = combine_fn(key, model)
    _, it = key_iter(key)
    if key == 0:
        return -1, None, np.zeros(n_corr, dtype=bool)
    return it, np.asarray(model).reshape(3, 3), mask_fn(model)


def point_shard(n, world, rank):
    """Contiguous point range of LinearTriangulation sharding (no collective:
    every range is independent; the caller gathers)."""
    return point_range(n, world, rank)


def allgather_torch(obj, group=None):
    """Every rank's obj, in rank order, over a torch.distributed group (gloo
    on the CPU tests; objects are small: point ranges, per-pair results)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def triangulate_sharded(tri_fn, x1, x2, world, rank, allgather):
    """LinearTriangulation over contiguous point ranges: this
    rank triangulates points [lo, hi) with tri_fn(x1[lo:hi], x2[lo:hi]) ->
    (hi - lo, 3); allgather(piece) returns every rank's piece in rank order.
    Points are independent, so the concatenation is the unsharded result."""
    lo, hi = point_shard(len(x1), world, rank)
    X = np.asarray(tri_fn(x1[lo:hi], x2[lo:hi]), dtype=np.float64).reshape(hi - lo, 3)
    return np.concatenate([np.asarray(p).reshape(-1, 3) for p in allgather(X)])


def f_ransac_from_table(core, points1, points2, index, samples, threshold=0.06):
    """get_inliers_ransac's result (Phase 1/GetInliersRANSAC.py:109-121) from
    a pre-drawn sample table (the draws happened elsewhere, in the stream's
    order).  samples is None when the reference would not draw (N < 8)."""
    index = np.asarray(index)
    if samples is None or len(samples) == 0:
        return None, np.array([])
    points1 = np.asarray(points1, dtype=np.float64).reshape(-1, 2)
    points2 = np.asarray(points2, dtype=np.float64).reshape(-1, 2)
    best, F, mask, _ = core.ransac_f8(points1, points2, samples, threshold)
    if best < 0:
        return None, np.array([])
    return F, index[np.where(mask)[0]]


def pair_loop_plan(pairs, f_points, homography, draw_table, n_max=1000):
    """The replicated part of pair_loop_spread: every pair's homography
    RANSAC and F sample table, in the driver's order, on the global stream.
    Returns [(H, h_idx, points1, points2, table or None)]."""
    n_iter = max(int(n_max), 0)
    plan = []
    for k, (x1, x2, index) in enumerate(pairs):
        H, h_idx = homography(x1, x2, index)
        p1, p2 = f_points(k, h_idx)
        n = len(p1)
        plan.append((H, h_idx, p1, p2, draw_table(n, n_iter) if (n >= 8 and n_iter > 0) else None))
    return plan


def pair_loop_local(plan, world, rank, f_ransac):
    """This rank's F-RANSACs: pairs k with k % world == rank -> {k: (F, f_idx)}."""
    return {k: f_ransac(p1, p2, h_idx, table)
            for k, (_, h_idx, p1, p2, table) in enumerate(plan) if k % world == rank}


def pair_loop_merge(plan, parts):
    """[(H, h_idx, F, f_idx)] for all pairs from every rank's local dict."""
    merged = {}
    for part in parts:
        merged.update(part)
    return [(H, h_idx) + tuple(merged[k]) for k, (H, h_idx, _, _, _) in enumerate(plan)]


def pair_loop_spread(pairs, f_points, world, rank, homography, draw_table, f_ransac, allgather, n_max=1000):
    """The pair loop of Wrapper_dev.py:67-123 with the F-RANSACs spread over
    ranks.

    pairs[k] = (x1, x2, index): pair k's homography inputs, in the driver's
    order.  f_points(k, h_idx) -> (points1, points2) of pair k's F-RANSAC.
    homography(x1, x2, index) -> (H, h_idx) consumes the global random stream
    (get_homography_inliers).  draw_table(N, n_iter) draws pair k's F table
    from the same stream exactly as GetInliersRANSAC's loop would
    (sample_table; nothing for N < 8 or n_iter = 0).  f_ransac(points1,
    points2, h_idx, table) -> (F, f_idx) scores it (f_ransac_from_table).
    Every rank runs the homography chain and draws every table -- so the
    stream leaves the loop where the sequential driver leaves it -- and
    scores the F-RANSACs of the pairs k with k % world == rank;
    allgather(dict) returns every rank's dict in rank order.  Returns
    [(H, h_idx, F, f_idx)] for all pairs."""
    plan = pair_loop_plan(pairs, f_points, homography, draw_table, n_max)
    return pair_loop_merge(plan, allgather(pair_loop_local(plan, world, rank, f_ransac)))
