"""bench.py's N > 1 control flow, end to end, on two gloo ranks on the CPU.

The driver runs `torchrun --nproc-per-node N bench.py --gpus N` on an 8-GPU
node; no GPU is available here, so the device calls bench.py makes through
`_sfmcore` are replaced by stand-ins and everything else is bench.py's own:
the process group, the unique-id broadcast, the point sharding
(sfm_dist.shard_ba), the barrier + max-over-ranks timing of the timed steps,
the hypothesis-sharded RANSAC (sfm_dist.ransac_sharded with the packed-key
combine), the rank-0-only JSON line and the teardown.  The stand-in BA solve
all-reduces a payload of the reduced camera system's size (36 nc (nc+1)/2 +
3 ns doubles) once per LM iteration over gloo, as the RCCL path
does; the stand-in RANSAC shard scores its hypotheses with the C oracle on the
table drawn from the global random stream.
"""
import contextlib
import io
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

STEPS, WARMUP, HYPS = 3, 1, 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _FakeCore:
    """The subset of _sfmcore bench.py calls, without a device."""

    def __init__(self, real):
        self.real = real
        self.iter_allreduces = 0
        self.single_solves = 0

    def require_device(self):
        pass

    class Comm:
        @staticmethod
        def unique_id():
            return b"u" * 128

        def __init__(self, uid, nranks, rank, device=None):
            assert len(uid) == 128 and nranks == dist.get_world_size() and rank == dist.get_rank()

        def close(self):
            pass

    def BAProblem(self, cams, pts, cam_idx, pt_idx, obs, K, comm=None, device=None):
        core = self

        class _BA:
            def __init__(self):
                nc = len(cams)
                self.payload = 36 * nc * (nc + 1) // 2 + 3 * 6 * nc
                self.n_obs = len(cam_idx)

            def solve(self, max_iterations=100, fixed_iterations=False, **_):
                for _ in range(max_iterations if comm is not None else 0):  # one all-reduce per iteration
                    t = torch.full((self.payload,), float(self.n_obs), dtype=torch.float64)
                    dist.all_reduce(t)
                    core.iter_allreduces += 1
                if comm is None:  # rank 0's single-rank re-solve (bench's multi_rank_check)
                    core.single_solves += 1
                return {"iterations": max_iterations, "accepted": min(5, max_iterations), "cost0": 2.0e5,
                        "cost": 1.0e5, "t_loop_ms": 0.5 * max_iterations, "status": 0}

            def download(self):  # the points of this problem, unchanged (the stand-in does not move them)
                return np.array(cams, dtype=np.float64), np.array(pts, dtype=np.float64)

            def reset(self):
                pass

            def set_timing(self, on=True):
                pass

            def kernel_times(self):
                return {"linearize": 0.01, "point_prep": 0.01, "schur_blocks": 0.05, "allreduce": 0.005,
                        "cholesky": 0.08, "backsub_trial": 0.02}

            def close(self):
                pass

        return _BA()

    def sample_table(self, n, k, H):
        return self.real.sample_table(n, k, H)

    def ransac_f8(self, x1, x2, samples, thr, device=None):
        return None

    def last_timings(self):
        return np.full(16, 0.01)

    def ransac_f8_range(self, x1, x2, H, h0, h1, thr, samples=None, want_counts=False, device=None):
        import oracle as O
        import sfm_dist
        table = self.real.sample_table(len(x1), 8, H)  # the whole table from the global stream, as the device call
        if h1 <= h0:
            return 0, np.zeros((3, 3)), None
        b, counts, F, _ = O.ransac(x1, x2, table[h0:h1], thr)
        return (sfm_dist.shard_key(counts[b], h0 + b) if b >= 0 else 0), F, None

    def ransac_f8_pyrandom(self, x1, x2, H, thr, want_counts=False, want_samples=False, device=None):
        import oracle as O
        table = self.real.sample_table(len(x1), 8, H)  # the global stream, as the device call draws it
        b, counts, F, m = O.ransac(x1, x2, table, thr)
        return b, (F if b >= 0 else None), m, None, None

    def ransac_combine(self, comm, key, M):
        import sfm_dist
        return sfm_dist.combine_keys_torch(key, M)

    def ransac_mask(self, x1, x2, M, thr, model=8, device=None):
        import oracle as O
        return O.ransac_mask(x1, x2, M, thr)


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, REPO)
    import bench
    import _sfmcore
    fake = _FakeCore(_sfmcore)
    bench.core = fake
    torch.cuda.is_available = lambda: True
    torch.cuda.set_device = lambda d: None
    torch.cuda.synchronize = lambda *a, **k: None
    sys.argv = ["bench.py", "--gpus", str(world), "--steps", str(STEPS), "--warmup", str(WARMUP), "--workload", "cfg3",
                "--no-secondary", "--no-next-rows", "--ransac-hyps", str(HYPS)]
    out = io.StringIO()
    try:
        with contextlib.redirect_stdout(out):
            bench.main()
        q.put((rank, out.getvalue(), fake.iter_allreduces, None, fake.single_solves))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, out.getvalue(), fake.iter_allreduces, repr(e), fake.single_solves))


def test_bench_two_rank_control_flow_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, text, n_ar, err, n_single = q.get(timeout=600)
        res[rank] = (text, n_ar, err, n_single)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r][2] is None, res[r][2]
    assert res[1][0].strip() == "", "only rank 0 prints the bench line"
    line = json.loads(res[0][0].strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["steps"] == STEPS and line["warmup"] == WARMUP
    assert line["unit"] == "LM-iterations/s" and line["scaling"] == "strong" and line["dtype"] == "f64"
    assert f"x{world}" in line["config"]["parallelism"] and f"over {world} rank(s)" in line["config"]["workload"]
    assert line["value"] > 0 and abs(line["ms_per_step"] - 1e3 * STEPS / line["value"] / STEPS) < 1e-3 * line["ms_per_step"] + 1e-3
    assert "end_to_end" not in line and "shard_local" not in line and "cpu_baseline" not in line  # N = 1 only
    ra = line["ransac"]
    assert ra["hypotheses"] == HYPS and "of 2" in ra["sharding"] and ra["hyps_per_s_end_to_end"] > 0
    assert ra["multi_rank_check"]["ok"] is True  # the sharded winner, F and mask are the unsharded call's
    # the converged solve (100), warmup, timed and timing runs each all-reduced once per iteration, on both ranks
    assert res[0][1] == res[1][1] == 100 + WARMUP + 2 * STEPS
    # the multi-rank check: rank 0 alone re-solves the whole problem once
    mc = line["multi_rank_check"]
    assert res[0][3] == 1 and res[1][3] == 0 and mc["ranks"] == world and mc["cost_spread_over_ranks"] == 0.0
    assert mc["sharded"]["iterations"] == mc["single_rank"]["iterations"] and mc["ok"] is True
