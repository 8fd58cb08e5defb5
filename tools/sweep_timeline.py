"""Dev probe: SFM_SWEEP_STAMPS stamps of the last k_schur_sweep launch of a
BA solve (cfg4 / cfg5): workgroup spans, dispatch waves, the prologue, per
chunk which side (pair waves or staging waves) reaches the barrier last,
and the end-of-range reduction."""
import os, sys, ctypes
os.environ["SFM_SWEEP_STAMPS"] = "1"
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R + '/structure-from-motion-_amd')
import numpy as np, _sfmcore as c, sfm_synthetic as syn
WG, EV, NW, NST = 4096, 68, 12, 2
name = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
p = syn.ba_problem_cfg(name, dense=False)
cams0 = np.column_stack([p["rotvec0"], np.einsum("nij,nj->ni", -p["R0"], p["C0"])])
prob = c.BAProblem(cams0, p["X0"], p["cam_idx"], p["pt_idx"], p["obs"], syn.K_REF)
prob.solve(max_iterations=2, fixed_iterations=True)
prob.close()
buf = np.zeros(WG * EV * NW, dtype=np.int64)
c._lib.sfm_sweep_debug(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), ctypes.c_int64(buf.size))
d = buf.reshape(WG, EV, NW).astype(np.float64)
used = np.where((d[:, 0, :] > 0).any(axis=1))[0]
d = d[used]
t0 = d[d > 0].min()
d = np.where(d > 0, (d - t0) * 0.01, np.nan)  # us
start = np.nanmin(d[:, 0, :], axis=1)
end = np.nanmax(d[:, EV - 1, :], axis=1)
span = end - start
print(f"{name}: {len(used)} workgroups; kernel span {np.nanmax(end):.1f} us; wg span mean {np.nanmean(span):.1f} "
      f"min {np.nanmin(span):.1f} max {np.nanmax(span):.1f}")
print("dispatch starts (us) quantiles:", np.round(np.nanquantile(start, [0, .1, .25, .5, .75, .9, 1]), 1))
print("ends (us) quantiles:", np.round(np.nanquantile(end, [0, .1, .25, .5, .75, .9, 1]), 1))
grp = d[:, :, :NW - NST]
stg = d[:, :, NW - NST:]
pro_s = np.nanmax(stg[:, 1, :], axis=1) - start
print(f"prologue (first chunk staged) mean {np.nanmean(pro_s):.1f} us")
w_grp, w_stg, nchunk, chunk_t = 0.0, 0.0, 0, []
last_chunk = np.full(len(used), np.nan)
for e in range(2, EV - 1):
    g_max = np.nanmax(grp[:, e, :], axis=1)
    g_min = np.nanmin(grp[:, e, :], axis=1)
    s_max = np.nanmax(stg[:, e, :], axis=1)
    ok = ~np.isnan(g_max) & ~np.isnan(s_max)
    if not ok.any():
        continue
    nchunk += ok.sum()
    w_grp += np.nansum(np.maximum(0, s_max - g_max)[ok])   # pair waves wait for the stagers
    w_stg += np.nansum(np.maximum(0, g_max - s_max)[ok])   # stagers wait for the pair waves
    chunk_t.append(np.nanmean((g_max - g_min)[ok]))
    last_chunk = np.where(ok, np.fmax(g_max, s_max), last_chunk)
print(f"chunks {nchunk} ({nchunk / len(used):.1f} per wg); pair waves wait for stagers {w_grp / nchunk:.2f} us/chunk, "
      f"stagers wait for pair waves {w_stg / nchunk:.2f} us/chunk; pair-wave spread (slowest - fastest) "
      f"{np.mean(chunk_t):.2f} us/chunk")
first = np.nanmax(d[:, 1, :], axis=1)
print(f"per wg: start->first staged {np.nanmean(first - start):.1f}, chunks {np.nanmean(last_chunk - first):.1f}, "
      f"reduction {np.nanmean(end - last_chunk):.1f} us")
