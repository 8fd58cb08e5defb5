"""Two RCCL ranks on ONE GPU (round 6 probe for VERDICT round 5 weak #9):
the BA's one-process-per-GPU transport with world size 2, both processes on
device 0.  Each rank solves its point shard (sfm_dist.shard_ba) through
core.Comm + BAProblem; rank 0 then solves the whole problem alone and
compares (iterations, accepted, cost, points).  The uid travels over a gloo
group.  Usage: python tools/rccl_two_ranks.py  (spawns the two ranks)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "structure-from-motion-_amd"))


def rank_main(rank, world, port):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import _sfmcore as core
    import sfm_dist
    import sfm_synthetic as syn
    p = syn.ba_problem(8, 3000, 4, seed=8, dense=False)
    cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
    uid = [core.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = core.Comm(uid[0], world, rank, device=0)
    ci, pi, ob, X, (lo, hi) = sfm_dist.shard_ba(p["cam_idx"], p["pt_idx"], p["obs"], p["X0"], world, rank)
    prob = core.BAProblem(cams0, X, ci, pi, ob, syn.K_REF, comm=comm, device=0)
    rep = prob.solve(max_iterations=30)
    c1, x1 = prob.download()
    prob.close()
    comm.close()
    parts = [None] * world
    dist.all_gather_object(parts, (lo, hi, x1, c1, rep))
    if rank == 0:
        X = np.concatenate([q[2] for q in sorted(parts, key=lambda q: q[0])])
        c0, x0, rep0 = core.ba_lm(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF, max_iterations=30)
        print("ranks", [q[4]["n_ranks"] for q in parts], "iterations", [q[4]["iterations"] for q in parts],
              "single", rep0["iterations"], "accepted", [q[4]["accepted"] for q in parts], rep0["accepted"],
              flush=True)
        print("cost", [q[4]["cost"] for q in parts], rep0["cost"], "max |X - X1|", float(np.abs(X - x0).max()),
              "max |c - c1|", float(np.abs(parts[0][3] - c0).max()), flush=True)
        ok = (all(q[4]["iterations"] == rep0["iterations"] for q in parts)
              and abs(parts[0][4]["cost"] - rep0["cost"]) <= 1e-9 * rep0["cost"]
              and np.abs(X - x0).max() <= 1e-8 * max(1.0, np.abs(x0).max()))
        print("RCCL_TWO_RANKS", "OK" if ok else "MISMATCH", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(rank_main, args=(2, port), nprocs=2, join=True, start_method="spawn")
