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
* LinearTriangulation: contiguous point ranges, no collective.
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
