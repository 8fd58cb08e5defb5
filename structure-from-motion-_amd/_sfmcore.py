"""ctypes binding of libsfmcore.so (include/sfmcore.h) for the drop-in modules.

This is the only route to compute: there is no CPU fallback.  Importing this
module fails loudly if the HIP library has not been built, and every compute
call raises ``SfmCoreError`` if no MI355X is visible.

The device is ``$SFM_DEVICE`` (default 0).
"""
import array
import ctypes
import os
import random

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsfmcore.so")


class SfmCoreError(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError(f"libsfmcore.so not built at {LIB_PATH}: run `make -C {_HERE}` "
                      "(or __graft_entry__.build()); there is no CPU fallback")

_lib = ctypes.CDLL(LIB_PATH)

_d = ctypes.POINTER(ctypes.c_double)
_i32 = ctypes.POINTER(ctypes.c_int32)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_i64 = ctypes.POINTER(ctypes.c_int64)
_u8 = ctypes.POINTER(ctypes.c_uint8)
_u64 = ctypes.POINTER(ctypes.c_uint64)
_c = ctypes.c_int
_i = ctypes.c_int64
_v = ctypes.c_void_p


class BAOpts(ctypes.Structure):
    _fields_ = [("max_iterations", ctypes.c_int32), ("fixed_iterations", ctypes.c_int32),
                ("function_tolerance", ctypes.c_double), ("gradient_tolerance", ctypes.c_double),
                ("parameter_tolerance", ctypes.c_double), ("initial_lambda", ctypes.c_double)]


class BAReport(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("accepted", ctypes.c_int32), ("status", ctypes.c_int32),
                ("n_ranks", ctypes.c_int32), ("cost0", ctypes.c_double), ("cost", ctypes.c_double),
                ("t_setup_ms", ctypes.c_double), ("t_loop_ms", ctypes.c_double),
                ("t_download_ms", ctypes.c_double), ("lambda_", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# (name, restype, argtypes) -- every symbol include/sfmcore.h declares
SIGNATURES = [
    ("sfm_version", _c, []),
    ("sfm_last_error", ctypes.c_char_p, []),
    ("sfm_device_count", _c, []),
    ("sfm_last_timings", _c, [_d, _c]),
    ("sfm_set_call_timing", _c, [_c]),
    ("sfm_pyrandom_sample_table", _c, [_u32, _i, ctypes.c_int32, _i, _i32]),
    ("sfm_f8_batch", _c, [_d, _d, _i, _d, _c]),
    ("sfm_f8_general", _c, [_d, _d, _i, _d, _c]),
    ("sfm_ransac_f8", _c, [_d, _d, _i, _i32, _i, ctypes.c_double, _i32, _i64, _d, _u8, _c]),
    # the in-call-sampling entries take raw addresses (c_void_p): the drop-in
    # calls them once per image pair and .ctypes.data_as costs ~4 us a pointer
    ("sfm_ransac_f8_pyrandom", _c, [_v, _v, _i, _v, _i, ctypes.c_double, _v, _v, _v, _v, _v, _c]),
    ("sfm_ransac_f8_dropin", _c, [_v, _v, _i, _v, _i, ctypes.c_double, _v, _v, _v, _v, _c]),
    ("sfm_ransac_f8_range", _c, [_d, _d, _i, _i32, _i, _i, _i, ctypes.c_double, _i32, _u64, _d, _c]),
    ("sfm_ransac_f8_pyrandom_range", _c, [_d, _d, _i, _u32, _i, _i, _i, ctypes.c_double, _i32, _u64, _d, _c]),
    ("sfm_ransac_f8_mask", _c, [_d, _d, _i, _d, ctypes.c_double, _u8, _c]),
    ("sfm_ransac_h4_pyrandom_range", _c, [_d, _d, _i, _u32, _i, _i, _i, ctypes.c_double, _i32, _u64, _d, _c]),
    ("sfm_ransac_h4_mask", _c, [_d, _d, _i, _d, ctypes.c_double, _u8, _c]),
    ("sfm_ransac_combine", _c, [ctypes.c_void_p, _u64, _d]),
    ("sfm_h4_batch", _c, [_d, _d, _i, _d, _c]),
    ("sfm_homography_general", _c, [_d, _d, _i, _d, _c]),
    ("sfm_ransac_h4", _c, [_d, _d, _i, _i32, _i, ctypes.c_double, _i32, _i64, _d, _u8, _c]),
    ("sfm_ransac_h4_pyrandom", _c, [_v, _v, _i, _v, _i, ctypes.c_double, _v, _v, _v, _v, _v, _c]),
    ("sfm_linear_pnp", _c, [_d, _d, _i, _d, _d, _d, _i32, _c]),
    ("sfm_pnp_ransac", _c, [_d, _d, _i, _d, _i32, _i, ctypes.c_double, _i32, _i32, _i64, _i64, _d, _d, _c]),
    ("sfm_nonlinear_pnp", _c, [_d, _d, _i, _d, _d, _d, ctypes.c_int32, _d, _d, _i32, _c]),
    ("sfm_matching_parse", _c, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p),
                                _i64, _i64]),
    ("sfm_matching_read", _c, [ctypes.c_void_p, _i32, _i32, _d, _d]),
    ("sfm_matching_free", _c, [ctypes.c_void_p]),
    ("sfm_dense_obs_scan", _c, [ctypes.c_void_p, ctypes.c_int32, _i, _i, _i64, _i, ctypes.c_int32, _d, _d, _i,
                                ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p), _i64]),
    ("sfm_dense_obs_read", _c, [ctypes.c_void_p, _i32, _i32, _d]),
    ("sfm_dense_obs_free", _c, [ctypes.c_void_p]),
    ("sfm_gather_rows3", _c, [_d, _i, _i64, _i, _d]),
    ("sfm_matrix_to_rotvec", ctypes.c_int64, [_d, _i, _d]),
    ("sfm_rotvec_to_matrix", _c, [_d, _i, _d]),
    ("sfm_triangulate_dlt", _c, [_d, _d, _d, _d, _i, _d, _c]),
    ("sfm_triangulate_nonlinear", _c, [_d, _d, _d, _d, _d, _i, ctypes.c_int32, _d, _i32, _c]),
    ("sfm_project_points", _c, [_d, _d, _i, _d, _c]),
    ("sfm_reduced_solve", _c, [_d, _d, ctypes.c_int32, _d, _c]),
    ("sfm_ba_residuals", _c, [ctypes.c_int32, _i, _i, _i32, _i32, _d, _d, _d, _d, _d, _c]),
    ("sfm_ba_lm", _c, [ctypes.c_int32, _i, _i, _i32, _i32, _d, _d, _d, _d, ctypes.POINTER(BAOpts),
                       ctypes.POINTER(BAReport), _c]),
    ("sfm_ba_lm_dense", _c, [ctypes.c_void_p, ctypes.c_int32, _i, _d, _d, _d, ctypes.POINTER(BAOpts),
                             ctypes.POINTER(BAReport), _c]),
    ("sfm_comm_unique_id", _c, [ctypes.c_char_p]),
    ("sfm_comm_init", _c, [ctypes.c_char_p, _c, _c, _c, ctypes.POINTER(ctypes.c_void_p)]),
    ("sfm_comm_init_local", _c, [_c, ctypes.POINTER(ctypes.c_void_p)]),
    ("sfm_comm_destroy", _c, [ctypes.c_void_p]),
    ("sfm_ba_create", _c, [ctypes.c_int32, _i, _i, _i32, _i32, _d, _d, _d, _d, _c, ctypes.c_void_p,
                           ctypes.POINTER(ctypes.c_void_p)]),
    ("sfm_ba_solve", _c, [ctypes.c_void_p, ctypes.POINTER(BAOpts), ctypes.POINTER(BAReport)]),
    ("sfm_ba_reset", _c, [ctypes.c_void_p]),
    ("sfm_ba_plan_digest", _c, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("sfm_ba_download", _c, [ctypes.c_void_p, _d, _d]),
    ("sfm_ba_kernel_times", _c, [ctypes.c_void_p, _d, _c, ctypes.c_char_p, _c]),
    ("sfm_ba_set_timing", _c, [ctypes.c_void_p, _c]),
    ("sfm_ba_destroy", _c, [ctypes.c_void_p]),
    ("sfm_ba_lm_multi", _c, [ctypes.c_int32, _i, _i, _i32, _i32, _d, _d, _d, _d, ctypes.POINTER(BAOpts),
                             ctypes.POINTER(BAReport), ctypes.POINTER(ctypes.c_int), _c]),
]
for _name, _res, _args in SIGNATURES:
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

DEVICE = int(os.environ.get("SFM_DEVICE", "0"))


def version():
    return _lib.sfm_version()


def device_count():
    return _lib.sfm_device_count()


_DEVICE_SEEN = False


def require_device():
    """Fail loudly without a HIP device (no CPU fallback); once a device has
    been seen the check is skipped (~2 us of a 0.19-ms RANSAC call)."""
    global _DEVICE_SEEN
    if _DEVICE_SEEN:
        return
    if _lib.sfm_device_count() <= 0:
        raise SfmCoreError("libsfmcore: no HIP device visible (the MI355X path has no CPU fallback)")
    _DEVICE_SEEN = True


def _check(rc):
    if rc != 0:
        raise SfmCoreError(f"libsfmcore error {rc}: {_lib.sfm_last_error().decode(errors='replace')}")


def _p(a, t=_d):
    return a.ctypes.data_as(t)


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def set_call_timing(on=True):
    """Device-side timings (HIP events) in the drop-in RANSAC calls."""
    _check(_lib.sfm_set_call_timing(int(bool(on))))


def last_timings():
    out = np.zeros(12)
    n = _lib.sfm_last_timings(_p(out), 12)
    return out[:n]


# ------------------------------------------------------------------ random
assert array.array("I").itemsize == 4

# The global generator's MT19937 state crosses the C-ABI as uint32[625] (624
# key words + position).  CPython keeps it inside the _random.Random object
# as {PyObject_HEAD; int index; uint32_t state[624]}; when import verifies
# that layout against random.getstate() (at three positions, one across a
# twist, and a write-back), the state is copied out of and back into the
# object with two memmoves -- random.getstate / setstate build and parse a
# 625-int tuple, ~25 us of every RANSAC drop-in call.  Otherwise (another
# interpreter, another layout) getstate / setstate.
_MT_INDEX = ctypes.sizeof(ctypes.c_ssize_t) + ctypes.sizeof(ctypes.c_void_p)  # after PyObject_HEAD
_MT_KEY = _MT_INDEX + 4
_MT_ZERO = bytes(625 * 4)


def _mt_layout_ok():
    import sys
    try:
        import _random
        inst = random.sample.__self__
        if (sys.implementation.name != "cpython" or not isinstance(inst, _random.Random)
                or _random.Random.__basicsize__ < _MT_KEY + 624 * 4):
            return False
    except (AttributeError, ImportError):
        return False
    saved = random.getstate()
    try:
        v, st, g = saved
        random.setstate((v, st[:624] + (623,), g))
        base = id(inst)
        for _ in range(3):  # positions 623, 624, then 1 after the twist
            _, cur, _ = random.getstate()
            raw = (ctypes.c_uint32 * 624).from_address(base + _MT_KEY)
            if tuple(raw) != cur[:624] or ctypes.c_int.from_address(base + _MT_INDEX).value != cur[624]:
                return False
            random.getrandbits(32)
        ctypes.c_int.from_address(base + _MT_INDEX).value = 5  # write-back
        return random.getstate()[1][624] == 5
    finally:
        random.setstate(saved)


_MT_DIRECT = _mt_layout_ok()


def _mt_state():
    """The global MT19937 state as a C uint32[625] (key + position) plus what
    _mt_restore needs to put it back (array.array: ~3x cheaper than numpy
    for the 625-int round trip of the getstate path)."""
    if _MT_DIRECT:
        base = id(random.sample.__self__)
        st = array.array("I", _MT_ZERO)
        ctypes.memmove(st.buffer_info()[0], base + _MT_KEY, 624 * 4)
        st[624] = ctypes.c_int.from_address(base + _MT_INDEX).value
        return base, st, None
    version_, internal, gauss = random.getstate()
    return version_, array.array("I", internal), gauss


def _mt_ptr(st):
    return ctypes.cast(st.buffer_info()[0], _u32)


def _mt_restore(h, st, gauss):
    if _MT_DIRECT:
        ctypes.memmove(h + _MT_KEY, st.buffer_info()[0], 624 * 4)
        ctypes.c_int.from_address(h + _MT_INDEX).value = st[624]
        return
    random.setstate((h, tuple(st), gauss))


def sample_table(n, k, H):
    """H draws of random.sample(range(n), k) on the GLOBAL random instance,
    replayed natively; the global state is advanced exactly as the
    reference's loop (GetInliersRANSAC.py:53-55) would advance it."""
    version_, st, gauss = _mt_state()
    out = np.empty((H, k), dtype=np.int32)
    _check(_lib.sfm_pyrandom_sample_table(_mt_ptr(st), int(n), int(k), int(H), _p(out, _i32)))
    _mt_restore(version_, st, gauss)
    return out


# --------------------------------------------------------------- geometry
def f8_batch(x1s, x2s):
    """H independent 8-point F estimates; x1s, x2s: (H, 8, 2)."""
    require_device()
    x1s, x2s = _f64(x1s), _f64(x2s)
    H = x1s.shape[0]
    F = np.zeros((H, 9))
    _check(_lib.sfm_f8_batch(_p(x1s), _p(x2s), H, _p(F), DEVICE))
    return F.reshape(H, 3, 3)


def f8_general(x1, x2):
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    F = np.zeros(9)
    _check(_lib.sfm_f8_general(_p(x1), _p(x2), len(x1), _p(F), DEVICE))
    return F.reshape(3, 3)


def ransac_f8(x1, x2, samples, thr, want_counts=False, device=None):
    """Returns (best_iter or -1, F_best (3,3) or None, mask (N,) bool, counts or None)."""
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    samples = np.ascontiguousarray(samples, dtype=np.int32)
    N, H = len(x1), len(samples)
    counts = np.zeros(H, dtype=np.int32) if want_counts else None
    best = np.zeros(1, dtype=np.int64)
    F = np.zeros(9)
    mask = np.zeros(N, dtype=np.uint8)
    _check(_lib.sfm_ransac_f8(_p(x1), _p(x2), N, _p(samples, _i32), H, float(thr),
                              _p(counts, _i32) if want_counts else None, _p(best, _i64), _p(F),
                              _p(mask, _u8), DEVICE if device is None else device))
    b = int(best[0])
    if b < 0:
        return -1, None, np.zeros(N, dtype=bool), counts
    return b, F.reshape(3, 3), mask.astype(bool), counts


def _ransac_pyrandom(fn, x1, x2, H, thr, want_counts, want_samples, device):
    """Shared body of the in-call-sampling RANSAC entries: the GLOBAL random
    state goes in, comes back advanced as H random.sample draws would."""
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    N = len(x1)
    version_, st, gauss = _mt_state()
    counts = np.zeros(H, dtype=np.int32) if want_counts else None
    samples = np.zeros((H, fn[1]), dtype=np.int32) if want_samples else None
    best = np.zeros(1, dtype=np.int64)
    M = np.zeros(9)
    mask = np.zeros(N, dtype=bool)  # written as 0/1 bytes by the library
    _check(fn[0](x1.ctypes.data, x2.ctypes.data, N, st.buffer_info()[0], int(H), float(thr),
                 counts.ctypes.data if want_counts else None, best.ctypes.data, M.ctypes.data, mask.ctypes.data,
                 samples.ctypes.data if want_samples else None, DEVICE if device is None else device))
    _mt_restore(version_, st, gauss)
    b = int(best[0])
    if b < 0:
        return -1, None, np.zeros(N, dtype=bool), counts, samples
    return b, M.reshape(3, 3), mask, counts, samples


def ransac_f8_pyrandom(x1, x2, H, thr, want_counts=False, want_samples=False, device=None):
    """GetInliersRANSAC's whole loop with the H 8-point samples drawn inside
    the call from the global random stream (sfm_ransac_f8_pyrandom).
    Returns (best_iter or -1, F_best or None, mask, counts or None, samples or None)."""
    return _ransac_pyrandom((_lib.sfm_ransac_f8_pyrandom, 8), x1, x2, H, thr, want_counts, want_samples, device)


def ransac_f8_dropin(x1, x2, H, thr, device=None):
    """GetInliersRANSAC's loop as its drop-in needs it (sfm_ransac_f8_dropin):
    (best_iter or -1, F_best or None, split, n_inliers) -- split[:n_inliers]
    the winner's inlier positions, split[n_inliers:] the outliers'."""
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    N = len(x1)
    h, st, gauss = _mt_state()
    out = np.zeros(2, dtype=np.int64)  # best_iter, n_inliers
    M = np.empty(9)
    split = np.empty(N, dtype=np.int64)
    oa = out.ctypes.data
    _check(_lib.sfm_ransac_f8_dropin(x1.ctypes.data, x2.ctypes.data, N, st.buffer_info()[0], int(H), float(thr), oa,
                                     M.ctypes.data, split.ctypes.data, oa + 8, DEVICE if device is None else device))
    _mt_restore(h, st, gauss)
    b = int(out[0])
    if b < 0:
        return -1, None, split[:0], 0
    return b, M.reshape(3, 3), split, int(out[1])


def ransac_h4_pyrandom(x1, x2, H, thr, want_counts=False, want_samples=False, device=None):
    """get_homography_inliers' loop with in-call sampling (sfm_ransac_h4_pyrandom)."""
    return _ransac_pyrandom((_lib.sfm_ransac_h4_pyrandom, 4), x1, x2, H, thr, want_counts, want_samples, device)


# ------------------------------------------- hypothesis-sharded RANSAC (§8(e))
def _ransac_range(model, x1, x2, H, h0, h1, thr, samples=None, want_counts=False, device=None):
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    N = len(x1)
    counts = np.zeros(max(h1 - h0, 0), dtype=np.int32) if want_counts else None
    key = np.zeros(1, dtype=np.uint64)
    M = np.zeros(9)
    dev = DEVICE if device is None else device
    cp = _p(counts, _i32) if want_counts else None
    if samples is not None:
        assert model == 8, "a given sample table is supported for the F model"
        samples = np.ascontiguousarray(samples, dtype=np.int32)
        assert samples.shape == (H, 8)
        _check(_lib.sfm_ransac_f8_range(_p(x1), _p(x2), N, _p(samples, _i32), int(H), int(h0), int(h1), float(thr),
                                        cp, _p(key, _u64), _p(M), dev))
    else:
        fn = _lib.sfm_ransac_f8_pyrandom_range if model == 8 else _lib.sfm_ransac_h4_pyrandom_range
        version_, st, gauss = _mt_state()
        _check(fn(_p(x1), _p(x2), N, _mt_ptr(st), int(H), int(h0), int(h1), float(thr), cp, _p(key, _u64), _p(M), dev))
        _mt_restore(version_, st, gauss)
    return int(key[0]), M.reshape(3, 3), counts


def ransac_f8_range(x1, x2, H, h0, h1, thr, samples=None, want_counts=False, device=None):
    """One hypothesis shard [h0, h1) of an H-hypothesis F-RANSAC.  Without
    `samples` the whole table is drawn from the GLOBAL random stream (which
    ends where the unsharded call leaves it) and only the shard is scored.
    Returns (key, F of the shard winner, counts or None); key = count << 32 |
    (0xFFFFFFFF - iteration), 0 if no hypothesis has an inlier."""
    return _ransac_range(8, x1, x2, H, h0, h1, thr, samples, want_counts, device)


def ransac_h4_range(x1, x2, H, h0, h1, thr, want_counts=False, device=None):
    """Homography counterpart of ransac_f8_range (in-call sampling)."""
    return _ransac_range(4, x1, x2, H, h0, h1, thr, None, want_counts, device)


def ransac_mask(x1, x2, M, thr, model=8, device=None):
    """Inlier mask of one model (the winner's emit after the combine)."""
    require_device()
    x1, x2, M = _f64(x1), _f64(x2), _f64(M)
    mask = np.zeros(len(x1), dtype=np.uint8)
    fn = _lib.sfm_ransac_f8_mask if model == 8 else _lib.sfm_ransac_h4_mask
    _check(fn(_p(x1), _p(x2), len(x1), _p(M), float(thr), _p(mask, _u8), DEVICE if device is None else device))
    return mask.astype(bool)


def ransac_combine(comm, key, M):
    """Max of the ranks' keys over `comm` (RCCL or an in-process group) and
    the winner's model.  Returns (key, model)."""
    k = np.array([key], dtype=np.uint64)
    M = np.array(M, dtype=np.float64).reshape(9).copy()
    _check(_lib.sfm_ransac_combine(comm.h if hasattr(comm, "h") else comm, _p(k, _u64), _p(M)))
    return int(k[0]), M.reshape(3, 3)


def local_group(nranks):
    """An in-process rank group (sfm_comm_init_local): one handle per rank,
    for N host threads sharing one process (and possibly one GPU)."""
    hs = (ctypes.c_void_p * nranks)()
    _check(_lib.sfm_comm_init_local(nranks, hs))
    return [LocalComm(h, nranks, r) for r, h in enumerate(hs)]


class LocalComm:
    def __init__(self, h, nranks, rank):
        self.h = ctypes.c_void_p(h)
        self.nranks, self.rank = nranks, rank

    def close(self):
        if self.h:
            _lib.sfm_comm_destroy(self.h)
            self.h = ctypes.c_void_p()


def h4_batch(x1s, x2s):
    """H independent 4-point homographies; x1s, x2s: (H, 4, 2)."""
    require_device()
    x1s, x2s = _f64(x1s), _f64(x2s)
    H = x1s.shape[0]
    out = np.zeros((H, 9))
    _check(_lib.sfm_h4_batch(_p(x1s), _p(x2s), H, _p(out), DEVICE))
    return out.reshape(H, 3, 3)


def homography_general(x1, x2):
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    out = np.zeros(9)
    _check(_lib.sfm_homography_general(_p(x1), _p(x2), len(x1), _p(out), DEVICE))
    return out.reshape(3, 3)


def ransac_h4(x1, x2, samples, thr, want_counts=False, device=None):
    """Returns (best_iter or -1, H_best (3,3) or None, mask (N,) bool, counts or None)."""
    require_device()
    x1, x2 = _f64(x1), _f64(x2)
    samples = np.ascontiguousarray(samples, dtype=np.int32)
    N, H = len(x1), len(samples)
    counts = np.zeros(H, dtype=np.int32) if want_counts else None
    best = np.zeros(1, dtype=np.int64)
    Hb = np.zeros(9)
    mask = np.zeros(N, dtype=np.uint8)
    _check(_lib.sfm_ransac_h4(_p(x1), _p(x2), N, _p(samples, _i32), H, float(thr),
                              _p(counts, _i32) if want_counts else None, _p(best, _i64), _p(Hb),
                              _p(mask, _u8), DEVICE if device is None else device))
    b = int(best[0])
    if b < 0:
        return -1, None, np.zeros(N, dtype=bool), counts
    return b, Hb.reshape(3, 3), mask.astype(bool), counts


def linear_pnp(X, x, K):
    """Returns (C (3,), R (3,3), branch)."""
    require_device()
    X, x, K = _f64(np.reshape(X, (-1, 3))), _f64(np.reshape(x, (-1, 2))), _f64(K)
    C, R, br = np.zeros(3), np.zeros(9), np.zeros(1, dtype=np.int32)
    _check(_lib.sfm_linear_pnp(_p(X), _p(x), len(X), _p(K), _p(C), _p(R), _p(br, _i32), DEVICE))
    return C, R.reshape(3, 3), int(br[0])


def pnp_ransac(X, x, K, samples, thr, want_counts=False):
    """Returns (best_iter or -1, best_count, C, R, counts or None, branches or None)."""
    require_device()
    X, x, K = _f64(np.reshape(X, (-1, 3))), _f64(np.reshape(x, (-1, 2))), _f64(K)
    samples = np.ascontiguousarray(samples, dtype=np.int32)
    H = len(samples)
    counts = np.zeros(H, dtype=np.int32) if want_counts else None
    branches = np.zeros(H, dtype=np.int32) if want_counts else None
    best, bc = np.zeros(1, dtype=np.int64), np.zeros(1, dtype=np.int64)
    C, R = np.zeros(3), np.zeros(9)
    _check(_lib.sfm_pnp_ransac(_p(X), _p(x), len(X), _p(K), _p(samples, _i32), H, float(thr),
                               _p(counts, _i32) if want_counts else None,
                               _p(branches, _i32) if want_counts else None, _p(best, _i64), _p(bc, _i64),
                               _p(C), _p(R), DEVICE))
    return int(best[0]), int(bc[0]), C, R.reshape(3, 3), counts, branches


def nonlinear_pnp(X, x, K, C0, R0, max_nfev=100, want_flags=False):
    """Returns (C (3,), R (3,3), info) -- info MINPACK's code (-1: the
    reference's except path) -- and with want_flags the CholeskyQR flags
    (1: shifted pass-1 factor, a third pass ran; 2: a Gram factor failed)."""
    require_device()
    X, x, K = _f64(np.reshape(X, (-1, 3))), _f64(np.reshape(x, (-1, 2))), _f64(K)
    C0, R0 = _f64(np.reshape(C0, 3)), _f64(np.reshape(R0, (3, 3)))
    C, R, info = np.zeros(3), np.zeros(9), np.zeros(1, dtype=np.int32)
    _check(_lib.sfm_nonlinear_pnp(_p(X), _p(x), len(X), _p(K), _p(C0), _p(R0), int(max_nfev), _p(C), _p(R),
                                  _p(info, _i32), DEVICE))
    v = int(info[0])
    code, flags = (v & 0xff, v >> 8) if v >= 0 else (v, 0)
    return (C, R.reshape(3, 3), code, flags) if want_flags else (C, R.reshape(3, 3), code)


def parse_matching(data_path, no_of_images, n_threads=0):
    """Native matching-file reader (host threads, no device needed).
    Returns (n_features, feature, image, x, y) -- COO, feature-major."""
    h = ctypes.c_void_p()
    nf, no = np.zeros(1, dtype=np.int64), np.zeros(1, dtype=np.int64)
    _check(_lib.sfm_matching_parse(os.fsencode(str(data_path)), int(no_of_images), int(n_threads), ctypes.byref(h),
                                   _p(nf, _i64), _p(no, _i64)))
    try:
        n = int(no[0])
        feat, img = np.empty(n, dtype=np.int32), np.empty(n, dtype=np.int32)
        x, y = np.empty(n), np.empty(n)
        _check(_lib.sfm_matching_read(h, _p(feat, _i32), _p(img, _i32), _p(x), _p(y)))
    finally:
        _lib.sfm_matching_free(h)
    return int(nf[0]), feat, img, x, y


_DENSE_DTYPES = {np.dtype(np.float64): 0, np.dtype(np.float32): 1, np.dtype(np.int64): 2, np.dtype(np.int32): 3,
                 np.dtype(np.uint8): 4, np.dtype(np.bool_): 4}


class DenseScan:
    """The native dense -> COO scan kept in the library (sfm_dense_obs_scan):
    len() observations, .arrays() copies them out as (camera_indices,
    point_indices, points_2d), ba_lm_dense() solves from it without the
    arrays.  close() (or the context manager) hands the pieces back."""

    def __init__(self, handle, n):
        self.h, self.n = handle, n

    def __len__(self):
        return self.n

    def arrays(self):
        n = self.n
        cam, pt, obs = np.empty(n, dtype=np.int32), np.empty(n, dtype=np.int32), np.empty((n, 2))
        _check(_lib.sfm_dense_obs_read(self.h, _p(cam, _i32), _p(pt, _i32), _p(obs)))
        return cam, pt, obs

    def close(self):
        if self.h:
            _lib.sfm_dense_obs_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def dense_scan(flags, feature_x, feature_y, rows, n_cams, n_threads=0):
    """np.where(flags[rows][:, :n_cams] == 1) and the coordinates at the hits,
    scanned natively (host threads, no device): a DenseScan, or None when the
    matrices' layout or dtype is not one the scanner reads (the caller then
    takes the numpy expression).  n_threads: row jobs (0: the library's)."""
    f, fx, fy = np.asarray(flags), np.asarray(feature_x), np.asarray(feature_y)
    if (f.ndim != 2 or fx.ndim != 2 or fx.shape != fy.shape or f.shape[0] != fx.shape[0]
            or f.dtype not in _DENSE_DTYPES or fx.dtype != np.float64 or fy.dtype != np.float64
            or f.strides[1] != f.itemsize or fx.strides != fy.strides or fx.strides[1] != 8
            or min(f.shape[1], fx.shape[1]) < n_cams):
        return None
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    h = ctypes.c_void_p()
    no = np.zeros(1, dtype=np.int64)
    _check(_lib.sfm_dense_obs_scan(f.ctypes.data, _DENSE_DTYPES[f.dtype], f.strides[0], f.shape[0],
                                   _p(rows, _i64), len(rows),
                                   int(n_cams), fx.ctypes.data_as(_d), fy.ctypes.data_as(_d), fx.strides[0],
                                   int(n_threads), ctypes.byref(h), _p(no, _i64)))
    return DenseScan(h, int(no[0]))


def dense_observations(flags, feature_x, feature_y, rows, n_cams, n_threads=0):
    """Native dense -> COO scan (host threads, no device needed): the
    observations np.where(flags[rows][:, :n_cams] == 1) gives, in its order,
    with feature_x / feature_y at the hits.  Returns (camera_indices,
    point_indices, points_2d), or None when the matrices' layout or dtype is
    not one the scanner reads (the caller then takes the numpy expression)."""
    scan = dense_scan(flags, feature_x, feature_y, rows, n_cams, n_threads)
    if scan is None:
        return None
    with scan:
        return scan.arrays()


def gather_points(all_world_coords, rows):
    """np.asarray(all_world_coords, dtype=float64)[rows] for the BA drop-in's
    x0 (BundleAdjustment.py:196-197), gathered by the host pool when the array
    is a C-ordered float64 n x 3 one and every row is in range; otherwise the
    numpy expression (its conversions and its IndexError)."""
    a = np.asarray(all_world_coords)
    rows = np.asarray(rows)
    if (a.dtype != np.float64 or a.ndim != 2 or a.shape[1] != 3 or not a.flags.c_contiguous
            or rows.dtype != np.int64 or rows.ndim != 1 or not rows.flags.c_contiguous):
        return np.asarray(all_world_coords, dtype=np.float64)[rows]
    out = np.empty((len(rows), 3))
    if _lib.sfm_gather_rows3(a.ctypes.data_as(_d), a.shape[0], _p(rows, _i64), len(rows), _p(out)) != 0:
        return a[rows]  # an index out of range: numpy's IndexError
    return out


def matrix_to_rotvec(Rs):
    """Rotation.from_matrix(Rs).as_rotvec() for an (n, 3, 3) stack, with
    scipy's bits (csrc/rotations.cpp); scipy itself when a matrix is not
    orthogonal to within 1e-13 (scipy orthogonalises it first) or the input
    is not a C-ordered float64 stack."""
    R = np.asarray(Rs)
    if R.dtype == np.float64 and R.ndim == 3 and R.shape[1:] == (3, 3) and R.flags.c_contiguous:
        w = np.empty((len(R), 3))
        if _lib.sfm_matrix_to_rotvec(R.ctypes.data_as(_d), len(R), _p(w)) == 0:
            return w
    from scipy.spatial.transform import Rotation
    return Rotation.from_matrix(Rs).as_rotvec()


def rotvec_to_matrix(w):
    """Rotation.from_rotvec(w).as_matrix() for an (n, 3) array, with scipy's
    bits (csrc/rotations.cpp)."""
    w = np.ascontiguousarray(w, dtype=np.float64)
    if w.ndim != 2 or w.shape[1] != 3:
        from scipy.spatial.transform import Rotation
        return Rotation.from_rotvec(w).as_matrix()
    R = np.empty((len(w), 3, 3))
    _check(_lib.sfm_rotvec_to_matrix(_p(w), len(w), _p(R)))
    return R


def triangulate(P1, P2, x1, x2):
    require_device()
    P1, P2, x1, x2 = _f64(P1), _f64(P2), _f64(x1), _f64(x2)
    X = np.zeros((len(x1), 3))
    _check(_lib.sfm_triangulate_dlt(_p(P1), _p(P2), _p(x1), _p(x2), len(x1), _p(X), DEVICE))
    return X


def triangulate_nonlinear(P1, P2, x1, x2, X0, max_nfev=50):
    """Returns (X (N,3), info (N,) int32): MINPACK info, -1 = x0 kept."""
    require_device()
    P1, P2 = _f64(P1), _f64(P2)
    x1, x2 = _f64(np.reshape(x1, (-1, 2))), _f64(np.reshape(x2, (-1, 2)))
    X0 = _f64(np.reshape(X0, (-1, 3)))
    X = np.zeros((len(x1), 3))
    info = np.zeros(len(x1), dtype=np.int32)
    _check(_lib.sfm_triangulate_nonlinear(_p(P1), _p(P2), _p(x1), _p(x2), _p(X0), len(x1), int(max_nfev), _p(X),
                                          _p(info, _i32), DEVICE))
    return X, info


def reduced_solve(S, rhs):
    """Diagnostic: x = S^-1 rhs with the bundle adjuster's reduced-camera
    solver (k_assemble + tiled Cholesky + substitutions)."""
    require_device()
    S = _f64(np.asarray(S))
    rhs = _f64(np.asarray(rhs).reshape(-1))
    n = len(rhs)
    if S.shape != (n, n):
        raise ValueError("S must be n x n")
    x = np.zeros(n)
    _check(_lib.sfm_reduced_solve(_p(S), _p(rhs), n, _p(x), DEVICE))
    return x


def project(P, X):
    require_device()
    P, X = _f64(P), _f64(X)
    out = np.zeros((len(X), 2))
    _check(_lib.sfm_project_points(_p(P), _p(X), len(X), _p(out), DEVICE))
    return out


def ba_residuals(cams, pts, cam_idx, pt_idx, obs, K):
    require_device()
    cams, pts, obs, K = _f64(cams), _f64(pts), _f64(obs), _f64(K)
    ci = np.ascontiguousarray(cam_idx, dtype=np.int32)
    pi = np.ascontiguousarray(pt_idx, dtype=np.int32)
    r = np.zeros(2 * len(ci))
    _check(_lib.sfm_ba_residuals(len(cams), len(pts), len(ci), _p(ci, _i32), _p(pi, _i32), _p(obs), _p(K),
                                 _p(cams), _p(pts), _p(r), DEVICE))
    return r


def ba_opts(max_iterations=100, fixed_iterations=False, function_tolerance=1e-10, gradient_tolerance=0.0,
            parameter_tolerance=1e-12, initial_lambda=1e-4):
    return BAOpts(int(max_iterations), int(bool(fixed_iterations)), function_tolerance, gradient_tolerance,
                  parameter_tolerance, initial_lambda)


def _own(a, own):
    """a as a C-order float64 array the solve may overwrite: a itself when
    the caller hands it over (own=True and already that layout), else a copy."""
    b = _f64(a)
    return b if own and b is a else b.copy()


def ba_lm(cams, pts, cam_idx, pt_idx, obs, K, own=False, **opts):
    """Schur-complement LM on the GPU. Returns (cams, pts, report dict);
    own=True: cams / pts are the caller's to overwrite (no copies)."""
    require_device()
    cams, pts = _own(cams, own), _own(pts, own)
    obs, K = _f64(obs), _f64(K)
    ci = np.ascontiguousarray(cam_idx, dtype=np.int32)
    pi = np.ascontiguousarray(pt_idx, dtype=np.int32)
    o, rep = ba_opts(**opts), BAReport()
    _check(_lib.sfm_ba_lm(len(cams), len(pts), len(ci), _p(ci, _i32), _p(pi, _i32), _p(obs), _p(K), _p(cams),
                          _p(pts), ctypes.byref(o), ctypes.byref(rep), DEVICE))
    return cams, pts, rep.as_dict()


def ba_lm_dense(cams, pts, scan, K, own=False, **opts):
    """ba_lm with the observations of a DenseScan (sfm_ba_lm_dense): they go
    from the scan's pieces into the upload buffer, no COO arrays."""
    require_device()
    cams, pts = _own(cams, own), _own(pts, own)
    o, rep = ba_opts(**opts), BAReport()
    _check(_lib.sfm_ba_lm_dense(scan.h, len(cams), len(pts), _p(_f64(K)), _p(cams), _p(pts), ctypes.byref(o),
                                ctypes.byref(rep), DEVICE))
    return cams, pts, rep.as_dict()


def ba_lm_multi(cams, pts, cam_idx, pt_idx, obs, K, devices, **opts):
    """Single-process multi-GPU LM: points split over `devices` (repeats allowed)."""
    require_device()
    cams, pts = _f64(cams).copy(), _f64(pts).copy()
    obs, K = _f64(obs), _f64(K)
    ci = np.ascontiguousarray(cam_idx, dtype=np.int32)
    pi = np.ascontiguousarray(pt_idx, dtype=np.int32)
    dev = (ctypes.c_int * len(devices))(*devices)
    o, rep = ba_opts(**opts), BAReport()
    _check(_lib.sfm_ba_lm_multi(len(cams), len(pts), len(ci), _p(ci, _i32), _p(pi, _i32), _p(obs), _p(K), _p(cams),
                                _p(pts), ctypes.byref(o), ctypes.byref(rep), dev, len(devices)))
    return cams, pts, rep.as_dict()


class Comm:
    """RCCL communicator for the multi-GPU BA (one process per GPU)."""

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(_lib.sfm_comm_unique_id(buf))
        return buf.raw

    def __init__(self, uid, nranks, rank, device=None):
        require_device()
        self.h = ctypes.c_void_p()
        dev = DEVICE if device is None else device
        _check(_lib.sfm_comm_init(ctypes.c_char_p(bytes(uid)), nranks, rank, dev, ctypes.byref(self.h)))

    def close(self):
        if self.h:
            _lib.sfm_comm_destroy(self.h)
            self.h = ctypes.c_void_p()


class BAProblem:
    """Device-resident BA problem (uploaded once, iterated many times)."""

    def __init__(self, cams, pts, cam_idx, pt_idx, obs, K, comm=None, device=None):
        require_device()
        self.n_cams, self.n_pts = len(cams), len(pts)
        cams, pts, obs, K = _f64(cams), _f64(pts), _f64(obs), _f64(K)
        ci = np.ascontiguousarray(cam_idx, dtype=np.int32)
        pi = np.ascontiguousarray(pt_idx, dtype=np.int32)
        self.n_obs = len(ci)
        self.h = ctypes.c_void_p()
        dev = DEVICE if device is None else device
        _check(_lib.sfm_ba_create(self.n_cams, self.n_pts, self.n_obs, _p(ci, _i32), _p(pi, _i32), _p(obs),
                                  _p(K), _p(cams), _p(pts), dev, comm.h if comm is not None else None,
                                  ctypes.byref(self.h)))

    def solve(self, **opts):
        o, rep = ba_opts(**opts), BAReport()
        _check(_lib.sfm_ba_solve(self.h, ctypes.byref(o), ctypes.byref(rep)))
        return rep.as_dict()

    def reset(self):
        _check(_lib.sfm_ba_reset(self.h))

    def plan_digest(self):
        """Digest of the Schur sweep plan (create with SFM_PLAN_DIGEST=1; else 0)."""
        d = ctypes.c_uint64()
        _check(_lib.sfm_ba_plan_digest(self.h, ctypes.byref(d)))
        return d.value

    def download(self):
        cams = np.zeros((self.n_cams, 6))
        pts = np.zeros((self.n_pts, 3))
        _check(_lib.sfm_ba_download(self.h, _p(cams), _p(pts)))
        return cams, pts

    def set_timing(self, on=True):
        """Per-phase HIP events in the following solves (kernel_times)."""
        _check(_lib.sfm_ba_set_timing(self.h, int(bool(on))))

    def kernel_times(self):
        ms = np.zeros(16)
        names = ctypes.create_string_buffer(512)
        n = _lib.sfm_ba_kernel_times(self.h, _p(ms), 16, names, 512)
        return dict(zip(names.value.decode().split(";"), ms[:n].tolist()))

    def close(self):
        if self.h:
            _lib.sfm_ba_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
