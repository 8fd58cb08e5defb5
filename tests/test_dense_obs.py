"""The BA drop-in's dense -> COO step (BundleAdjustment.py:164-169): the
library's threaded scan (csrc/dense_obs.cpp) against the reference's numpy
expression, on the flag dtypes the reference's drivers build (int, float,
bool), with invalid rows, flags other than 0/1, a camera count below the
matrices' width and a row-strided view.  Host only (no device)."""
import numpy as np
import pytest

import _sfmcore as core
import BundleAdjustment as BA


def reference_observations(fwc, fx, fy, flags, n_cams):
    valid = np.where(np.asarray(fwc).flatten() == 1)[0]
    f = np.asarray(flags)[valid][:, :n_cams] == 1
    pi, ci = np.nonzero(f)
    rows = valid[pi]
    return valid, ci, pi, np.column_stack([np.asarray(fx)[rows, ci], np.asarray(fy)[rows, ci]])


def problem(n, m, dtype, seed):
    rng = np.random.default_rng(seed)
    flags = (rng.random((n, m)) < 0.2).astype(dtype)
    if np.dtype(dtype).kind in "fi":
        flags[rng.random((n, m)) < 0.02] = 2  # not == 1: no observation
    fx, fy = rng.standard_normal((n, m)), rng.standard_normal((n, m))
    fwc = (rng.random((n, 1)) < 0.8).astype(np.int64)
    return fwc, fx, fy, flags


@pytest.mark.parametrize("dtype", [np.int64, np.float64, np.int32, np.float32, np.bool_, np.uint8])
@pytest.mark.parametrize("n_threads", [0, 1, 3])
def test_dense_observations_match_numpy(dtype, n_threads):
    fwc, fx, fy, flags = problem(20011, 37, dtype, 7)
    n_cams = 33  # the reference slices [:, :n_cameras]
    valid, ci, pi, obs = reference_observations(fwc, fx, fy, flags, n_cams)
    got = core.dense_observations(flags, fx, fy, valid, n_cams, n_threads=n_threads)
    assert got is not None
    cam, pt, xy = got
    assert np.array_equal(cam, ci) and np.array_equal(pt, pi)
    assert np.array_equal(xy, obs)  # gathered, not computed: bit for bit


def test_drop_in_observations_equal_reference_and_fallback():
    fwc, fx, fy, flags = problem(5003, 20, np.int64, 11)
    ref = reference_observations(fwc, fx, fy, flags, 20)
    got = BA._observations(fwc, fx, fy, flags, 20)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    # a view the scanner does not read (column-strided): numpy's expression
    fx2 = np.asfortranarray(fx)
    assert core.dense_observations(flags, fx2, fy, ref[0], 20) is None
    for a, b in zip(BA._observations(fwc, fx2, fy, flags, 20), ref):
        assert np.array_equal(a, b)
    # a row-strided view (every other row of bigger matrices) is read in place
    big = [np.repeat(a, 2, axis=0) for a in (fx, fy, flags)]
    views = [a[::2] for a in big]
    for a, b in zip(BA._observations(fwc, *views, 20), ref):
        assert np.array_equal(a, b)


def test_dense_observations_empty():
    fwc, fx, fy, flags = problem(100, 5, np.int64, 3)
    cam, pt, xy = core.dense_observations(flags, fx, fy, np.zeros(0, dtype=np.int64), 5)
    assert len(cam) == len(pt) == len(xy) == 0
    flags[:] = 0
    cam, pt, xy = core.dense_observations(flags, fx, fy, np.arange(100), 5)
    assert len(cam) == 0 and xy.shape == (0, 2)


def test_dense_observations_row_out_of_bounds():
    """a valid row past the matrices is refused by the scan (no
    out-of-bounds host read), and the drop-in raises IndexError from the
    observation loop as the reference does (its loop is outside the try,
    BundleAdjustment.py:164-169)."""
    fwc, fx, fy, flags = problem(100, 5, np.int64, 3)
    with pytest.raises(core.SfmCoreError, match="out of bounds"):
        core.dense_observations(flags, fx, fy, np.array([3, 100]), 5)
    big = np.ones((120, 1), dtype=np.int64)  # 20 more valid rows than the matrices have
    R = [np.eye(3)] * 5
    C = [np.zeros(3)] * 5
    with pytest.raises(IndexError, match="out of bounds for axis 0 with size 100"):
        BA.perform_bundle_adjustment(np.zeros((120, 3)), big, fx, fy, flags, R, C, np.eye(3), 4)
    with pytest.raises(IndexError, match="axis 1"):  # more cameras than flag columns
        BA.perform_bundle_adjustment(np.zeros((100, 3)), fwc, fx, fy, flags, R + R, C + C, np.eye(3), 4)


def test_gather_points_equals_numpy_fancy_index():
    """The BA drop-in's x0 points (BundleAdjustment.py:196-197): the native
    gather equals np.asarray(a, float64)[rows] for every row pattern, falls
    back to numpy for other dtypes / layouts, and raises numpy's IndexError."""
    import _sfmcore as core
    rng = np.random.default_rng(4)
    a = rng.standard_normal((200_000, 3))
    for rows in (np.arange(len(a)), np.sort(rng.choice(len(a), 70_000, replace=False)), np.array([7], np.int64),
                 np.zeros(0, np.int64)):
        assert np.array_equal(core.gather_points(a, rows), a[rows])
    assert np.array_equal(core.gather_points(a.astype(np.float32), np.array([1, 2])),
                          a.astype(np.float32).astype(np.float64)[[1, 2]])
    assert np.array_equal(core.gather_points(np.asfortranarray(a), np.array([3, 9])), a[[3, 9]])
    with pytest.raises(IndexError):
        core.gather_points(a, np.array([len(a)], np.int64))


@pytest.mark.parametrize("job", [0, 5, 97])
def test_scan_exception_becomes_error_code(job, monkeypatch):
    """A host allocation failure inside a scan job (the caller's thread or a
    pool worker: jobs are dealt dynamically) comes back through the C-ABI as
    SFM_ERR_NOMEM with its reason, after every worker has left the job; the
    next scan runs normally (csrc/host_pool.hpp's exception contract)."""
    import _sfmcore as core
    rng = np.random.default_rng(4)
    n, c = 98 * 1024, 24
    flags = (rng.random((n, c)) < 0.3).astype(np.int64)
    fx, fy = rng.random((n, c)), rng.random((n, c))
    rows = np.arange(n, dtype=np.int64)
    monkeypatch.setenv("SFM_TEST_SCAN_THROW", str(job))
    with pytest.raises(core.SfmCoreError, match="host memory allocation failed"):
        core.dense_observations(flags, fx, fy, rows, c)
    monkeypatch.delenv("SFM_TEST_SCAN_THROW")
    cam, pt, obs = core.dense_observations(flags, fx, fy, rows, c)
    pi, ci = np.nonzero(flags == 1)
    assert np.array_equal(cam, ci) and np.array_equal(pt, pi) and np.array_equal(obs[:, 0], fx[pi, ci])


def test_scan_on_one_allowed_cpu_is_serial_and_equal():
    """the host passes size their threads from the process's
    affinity mask (csrc/host_pool.hpp host_threads), not the machine's CPU
    count.  A child pinned to one CPU runs the dense scan (256 jobs) on that
    one thread and gets numpy's observations."""
    import os
    import subprocess
    import sys
    if not hasattr(os, "sched_setaffinity"):
        pytest.skip("no affinity API")
    here = os.path.dirname(os.path.abspath(__file__))
    code = (
        "import os, sys, numpy as np\n"
        "os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})\n"
        f"sys.path.insert(0, {os.path.join(os.path.dirname(here), 'structure-from-motion-_amd')!r})\n"
        "import _sfmcore as core\n"
        "rng = np.random.default_rng(9)\n"
        "n, c = 98 * 1024, 24\n"
        "flags = (rng.random((n, c)) < 0.3).astype(np.int64)\n"
        "fx, fy = rng.random((n, c)), rng.random((n, c))\n"
        "before = len(os.listdir('/proc/self/task'))\n"
        "cam, pt, obs = core.dense_observations(flags, fx, fy, np.arange(n, dtype=np.int64), c)\n"
        "pi, ci = np.nonzero(flags == 1)\n"
        "assert np.array_equal(cam, ci) and np.array_equal(pt, pi) and np.array_equal(obs[:, 1], fy[pi, ci])\n"
        "tasks = len(os.listdir('/proc/self/task'))\n"
        "assert tasks == before, (before, tasks)  # no pool workers were spawned for one CPU\n"
    )
    env = dict(os.environ)
    env.pop("SFM_PLAN_THREADS", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
