"""Timeline (kernels + copies) of the last RANSAC call in a rocprofv3 trace
(tools/trace_ransac.sh).  Usage: python tools/ransac_timeline.py gpurun_out/<tag>/trace"""
import csv, glob, sys
d = sys.argv[1]
k = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
mf = glob.glob(d + "/*memory_copy_trace.csv")
m = list(csv.DictReader(open(mf[0]))) if mf else []
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sfm::", "")[:30]) for r in k]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"]) for r in m]
ev.sort()
sel = [i for i, e in enumerate(ev) if "select" in e[2]]
a = sel[-2] + 1
t0, prev = ev[a][0], None
for s, e, n in ev[a:]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {((s - prev) / 1e3 if prev else 0):6.1f}  {n}")
    prev = e
