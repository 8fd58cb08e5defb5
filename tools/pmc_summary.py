"""Summarise rocprofv3 runs into profiles/<round>/ (committed evidence).

  python tools/pmc_summary.py gpurun_out/<dir> profiles/round3 [ITERATIONS [WORKLOAD]]

<dir> holds: kernel_trace/ (rocprofv3 --kernel-trace --stats) and
FETCH_SIZE/, WRITE_SIZE/, TCC_HIT_sum_TCC_MISS_sum/ (separate --pmc passes).
Writes kernel_stats.csv (copy), kernel_stats.md and pmc_traffic.json with
per-launch averages per kernel.  HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) *
1024: FETCH_SIZE/WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE reports half
of a wide coalesced read (MI355X_MICROARCH.md, HBM section).
With ITERATIONS (the PMC passes profiled tools/ba_once.py running that many
LM iterations), also pmc_iteration.json: every kernel's bytes summed over
its launches / ITERATIONS -- the HBM traffic of one LM iteration (named
pmc_iteration_<WORKLOAD>.json when WORKLOAD is given; the other files then
carry the _<WORKLOAD> suffix too).  Any other pass directory (e.g. the FP64
VALU counters) lands in pmc_traffic as per-launch averages and totals.
"""
import collections
import csv
import json
import os
import shutil
import sys


# sfm_ba_create's device-side work (once per problem, not per LM iteration):
# the camera-major copies, the CSR / radix sort, the sweep planner's passes
SETUP_KERNELS = ("k_gather_cam_major", "k_csr_cnt", "k_csr_cnt_lds", "k_csr_pstart", "k_csr_cstart",
                 "k_plan_counts", "k_plan_counts_lds", "k_plan_chunkmax", "k_plan_chunkcnt", "k_plan_chunkmax_fin",
                 "k_plan_lists", "k_plan_narrow")


def is_setup(name):
    return short(name) in SETUP_KERNELS or "rocprim" in name


def short(name):
    return name.split("(")[0].replace("sfm::", "")


def main(src, dst, iterations=0, workload=""):
    os.makedirs(dst, exist_ok=True)
    sfx = f"_{workload}" if workload else ""
    ks = os.path.join(src, "kernel_trace", "run_kernel_stats.csv")
    out = {}
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, f"kernel_stats{sfx}.csv"))
        rows = list(csv.DictReader(open(ks)))
        with open(os.path.join(dst, f"kernel_stats{sfx}.md"), "w") as f:
            f.write("| kernel | calls | avg us | total ms | % |\n|---|---|---|---|---|\n")
            for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
                f.write(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                        f"{float(r['TotalDurationNs']) / 1e6:.3f} | {float(r['Percentage']):.1f} |\n")
    tags = sorted(t for t in os.listdir(src) if os.path.exists(os.path.join(src, t, "run_counter_collection.csv")))
    for tag in tags:
        f = os.path.join(src, tag, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in agg.items():
            for c, v in d.items():
                out.setdefault(k, {})[c] = sum(v) / len(v)
                out[k][c + "_total"] = sum(v)
                out[k]["launches"] = len(v)
    for k, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        if "TCC_HIT_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d.get("TCC_MISS_sum", 0))
    json.dump(out, open(os.path.join(dst, f"pmc_traffic{sfx}.json"), "w"), indent=1, sort_keys=True)
    if iterations:
        # create-time launches (once per problem, not per LM iteration) are
        # kept out of the per-iteration bytes and listed beside them
        setup = [k for k in out if is_setup(k)]
        per = {k: (2 * d["FETCH_SIZE_total"] + d["WRITE_SIZE_total"]) * 1024 / iterations
               for k, d in out.items() if "FETCH_SIZE_total" in d and "WRITE_SIZE_total" in d and k not in setup}
        json.dump({"iterations": iterations, "source": src, "total_bytes_per_iteration": sum(per.values()),
                   "bytes_per_iteration": per, "excluded_setup_kernels": setup},
                  open(os.path.join(dst, f"pmc_iteration{sfx}.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps({k: {c: round(v, 1) for c, v in d.items()} for k, d in out.items() if "k_" in k}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0,
         sys.argv[4] if len(sys.argv) > 4 else "")
