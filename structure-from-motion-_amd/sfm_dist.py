"""Multi-GPU partitioning of the hot path.

* BA: points -- with all of their observations -- are split into contiguous
  ranges, one per rank; every rank holds every camera.  Each observation
  lives on exactly one rank, so the per-rank partial reduced camera systems
  simply add (one RCCL all-reduce per LM iteration, csrc/ba.hip).
* RANSAC: hypotheses are split into contiguous ranges; the global winner is
  (max count, then min iteration), i.e. the reference's strict '>' rule
  applied across ranks.
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


def combine_ransac(per_rank):
    """per_rank: list of (best_count, best_global_iter or -1) -> (count, iter)."""
    best_c, best_i = 0, -1
    for c, i in per_rank:
        if i < 0 or c <= 0:
            continue
        if c > best_c or (c == best_c and i < best_i):
            best_c, best_i = c, i
    return best_c, best_i
