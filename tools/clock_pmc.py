"""Effective shader clock per kernel from a rocprofv3 `--pmc GRBM_GUI_ACTIVE
GRBM_COUNT --kernel-trace` run (MI355X_MICROARCH.md, DVFS give-back:
GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's wall time; reads high on dispatches
shorter than ~0.3 ms).  Usage: clock_pmc.py <run_counter_collection.csv>..."""
import csv, sys, collections
for path in sys.argv[1:]:
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        ns = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        if ns <= 0:
            continue
        name = row["Kernel_Name"].split("(")[0]
        acc[name].append((float(row["Counter_Value"]) / 8.0 / ns, ns / 1e3))
    print(path)
    for name, v in sorted(acc.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
        ghz = sorted(x[0] for x in v)
        us = sorted(x[1] for x in v)
        print(f"  {name[:60]:60s} n {len(v):4d}  median {us[len(us) // 2]:8.1f} us  clock {ghz[len(ghz) // 2]:.2f} GHz"
              f" (p10 {ghz[len(ghz) // 10]:.2f}, p90 {ghz[9 * len(ghz) // 10]:.2f})")
