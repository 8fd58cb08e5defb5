"""TEST INFRASTRUCTURE ONLY: pure-Python restatement of the reference's
get_data loop (Phase 1/Utils.py:8-64), the checker for the native matching
reader (structure-from-motion-_amd/csrc/matching_io.cpp).  Small inputs."""
import numpy as np


def get_data(data_path, no_of_images):
    xs, ys, fs = [], [], []
    for n in range(1, no_of_images):  # :23
        with open(f"{data_path}/matching{n}.txt", "r") as fh:
            for i, row in enumerate(fh):
                if i == 0:  # :27
                    continue
                xr = np.zeros(no_of_images)
                yr = np.zeros(no_of_images)
                fr = np.zeros(no_of_images, dtype=int)
                cols = np.asarray([float(t) for t in row.split()])
                left = cols[0]
                xr[n - 1], yr[n - 1], fr[n - 1] = cols[4], cols[5], 1  # :36-43
                m = 1
                while left > 1:  # :45-55
                    k = int(cols[5 + m])
                    xr[k - 1], yr[k - 1], fr[k - 1] = int(cols[6 + m]), int(cols[7 + m]), 1
                    m += 3
                    left = left - 1
                xs.append(xr)
                ys.append(yr)
                fs.append(fr)
    shape = (-1, no_of_images)
    return (np.asarray(xs).reshape(shape), np.asarray(ys).reshape(shape), np.asarray(fs).reshape(shape))
