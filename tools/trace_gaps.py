"""Timeline of a rocprofv3 kernel trace (tools/trace_conv.sh): per LM
iteration (k_lm_step ends one), each kernel's duration and the idle gap
before it.  Usage: python tools/trace_gaps.py gpurun_out/<tag>/trace"""
import csv, glob, sys
from collections import defaultdict

path = sys.argv[1]
f = glob.glob(path + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the traced (second) solve: from the last k_lm_reset on
resets = [i for i, r in enumerate(rows) if "k_lm_reset" in r["Kernel_Name"]]
rows = rows[resets[-1]:]
it, prev_end, t0 = 0, None, int(rows[0]["Start_Timestamp"])
per = defaultdict(lambda: [0.0, 0.0, 0])
line = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sfm::", "")
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    dur = (e - s) / 1e3
    per[name][0] += dur; per[name][1] += gap; per[name][2] += 1
    line.append(f"{name}:{dur:.1f}(+{gap:.1f})")
    prev_end = e
    if name.startswith("k_lm_step"):
        print(f"it {it}: " + " ".join(line))
        line, it = [], it + 1
if line:
    print("tail: " + " ".join(line))
print(f"total {(prev_end - t0) / 1e3:.1f} us over {it} iterations")
for k, (d, g, n) in sorted(per.items(), key=lambda x: -x[1][0]):
    print(f"{k:32s} n={n:4d} busy={d:8.1f} us gaps={g:8.1f} us avg={d / n:6.2f}")
