"""Native matching-file reader (csrc/matching_io.cpp) vs the reference's
get_data: the reference's own output on P3Data (tests/golden), and the
restated loop (oracle/matching.py) on synthetic files with the format's edge
cases.  Host-only code: runs in the CPU suite."""
import os

import numpy as np
import pytest

import oracle_matching as OM
import sfm_io
from conftest import GOLDEN


def test_get_data_matches_reference_on_p3data(golden):
    p = golden("ransac_p3data.npz")
    fx, fy, ff = sfm_io.get_data(os.path.join(GOLDEN, "P3Data"), 5)
    assert fx.dtype == p["feature_x"].dtype and ff.dtype == p["feature_flag"].dtype
    assert np.array_equal(fx, p["feature_x"]) and np.array_equal(fy, p["feature_y"])
    assert np.array_equal(ff, p["feature_flag"])


def _write_scene(d, n_img, rows_per_file, seed, edge=False):
    rng = np.random.default_rng(seed)
    for n in range(1, n_img):
        lines = [f"nFeatures: {rows_per_file}"]
        for r in range(rows_per_file):
            others = rng.choice(np.arange(n + 1, n_img + 1), size=rng.integers(0, n_img - n + 1), replace=False) \
                if n < n_img else []
            toks = [str(len(others) + 1), "255", "128", "0", repr(float(rng.uniform(0, 1280))),
                    repr(float(rng.uniform(0, 960)))]
            for o in others:
                toks += [str(int(o)), f"{rng.uniform(-5, 1280):.6f}", f"{rng.uniform(-5, 960):.5e}"]
            if edge and r % 7 == 0:
                toks[4] = "+" + toks[4]                      # leading '+'
                toks += []
            if edge and r % 11 == 0 and len(others):
                toks[0] = str(len(others) + 2)               # repeat the first match: last write wins
                toks += [str(int(others[0])), "17.9", "-3.2"]
            if edge and r % 13 == 0:
                toks[0] = str(int(toks[0]) + 1)              # image id 0 wraps to the last image
                toks += ["0", "5.5", "6.5"]
            sep = "\t" if (edge and r % 5 == 0) else " "
            lines.append(sep.join(toks) + (" \r" if edge and r % 3 == 0 else " "))
        with open(os.path.join(d, f"matching{n}.txt"), "w") as fh:
            fh.write("\n".join(lines) + "\n")


@pytest.mark.parametrize("edge", [False, True])
def test_reader_matches_restated_loop(tmp_path, edge):
    _write_scene(tmp_path, 6, 400, seed=3 + edge, edge=edge)
    ref = OM.get_data(str(tmp_path), 6)
    got = sfm_io.get_data(str(tmp_path), 6)
    for a, b in zip(got, ref):
        assert a.shape == b.shape and np.array_equal(a, b)


def test_reader_chunked_threads_equal_single_thread(tmp_path):
    _write_scene(tmp_path, 4, 30_000, seed=9)  # > 256 KiB per file: several chunks
    assert os.path.getsize(tmp_path / "matching1.txt") > 1 << 20
    one = sfm_io.read_matching(str(tmp_path), 4, n_threads=1)
    many = sfm_io.read_matching(str(tmp_path), 4, n_threads=8)
    for k in ("feature", "image", "x", "y"):
        assert np.array_equal(getattr(one, k), getattr(many, k))
    ref = OM.get_data(str(tmp_path), 4)
    for a, b in zip(many.dense(), ref):
        assert np.array_equal(a, b)


def test_store_observations_equal_dense_path(tmp_path):
    from BundleAdjustment import _observations
    _write_scene(tmp_path, 6, 300, seed=5)
    st = sfm_io.read_matching(str(tmp_path), 6)
    fx, fy, ff = st.dense()
    rng = np.random.default_rng(1)
    valid = (rng.random(st.n_features) < 0.6).astype(int).reshape(-1, 1)
    filt = np.zeros_like(ff)
    for img in range(6):  # filtered_feature_flags[rows, img] = 1, as the driver does
        rows = np.where(ff[:, img] & (rng.random(st.n_features) < 0.7))[0]
        filt[rows, img] = 1
        st.set_flags(rows, img)
    for n_cams in (3, 6):
        a = _observations(valid, fx, fy, filt, n_cams)
        b = st.observations(valid, n_cams)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_reader_errors(tmp_path):
    import _sfmcore
    with pytest.raises(_sfmcore.SfmCoreError, match="No such file"):
        sfm_io.get_data(str(tmp_path), 3)
    (tmp_path / "matching1.txt").write_text("nFeatures: 1\n2 1 2 3 4.0 5.0 2 7 abc\n")
    with pytest.raises(_sfmcore.SfmCoreError, match="could not convert"):
        sfm_io.get_data(str(tmp_path), 2)
    (tmp_path / "matching1.txt").write_text("nFeatures: 1\n3 1 2 3 4.0 5.0 2 7 8\n")
    with pytest.raises(_sfmcore.SfmCoreError, match="index out of range"):
        sfm_io.get_data(str(tmp_path), 3)
    (tmp_path / "matching1.txt").write_text("nFeatures: 0\n")
    fx, fy, ff = sfm_io.get_data(str(tmp_path), 2)
    assert fx.shape == (0, 2) and ff.shape == (0, 2)
