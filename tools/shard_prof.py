"""Rank 0's point shard of cfg5 for N ranks, alone on this GPU (one-rank RCCL
communicator, as bench.py shard_local), W + K fixed LM iterations: the
program to put under rocprofv3 --kernel-trace --stats for the per-kernel
split of the sharded step.  Usage: python tools/shard_prof.py N [K]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "structure-from-motion-_amd"),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]
import numpy as np  # noqa: E402
import _sfmcore as core  # noqa: E402
import sfm_dist  # noqa: E402
import sfm_synthetic as syn  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
K3 = syn.K_REF
prob = syn.ba_problem_cfg("cfg5", dense=False)
cams0 = np.column_stack([prob["rotvec0"], np.einsum("nij,nj->ni", -prob["R0"], prob["C0"])])
comm = core.Comm(core.Comm.unique_id(), 1, 0, device=0)
ci, pi, ob, X0, _ = sfm_dist.shard_ba(prob["cam_idx"], prob["pt_idx"], prob["obs"], prob["X0"], n, 0)
ba = core.BAProblem(cams0, X0, ci, pi, ob, K3, comm=comm)
ba.solve(max_iterations=3, fixed_iterations=True)
ba.reset()
ba.set_timing(True)
ba.solve(max_iterations=K, fixed_iterations=True)
print({k: round(v, 4) for k, v in ba.kernel_times().items()})
ba.close()
comm.close()
