"""Kernel sequence of one adaptive step from a rocprofv3 kernel + HIP
runtime trace of tools/adapt_loop.py (steps start at k_adapt_diff), with
each kernel's duration and the idle gap before it: where the device waits
for the host.  usage: python tools/step_seq.py <trace dir> [step from the end]"""
import csv
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kt = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
api = {r["Correlation_Id"]: r["Function"] for r in tr}
kt.sort(key=lambda k: int(k["Start_Timestamp"]))
idx = [i for i, k in enumerate(kt) if ("k_adapt_diff" in k["Kernel_Name"] or "k_adapt_faces" in k["Kernel_Name"])]
a, b = idx[-back], idx[-back + 1]
prev = None
busy = gaps = 0
for k in kt[a:b]:
    n = k["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-50:]
    s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    prev = e
    busy += (e - s) / 1e3
    gaps += max(gap, 0)
    print(f"{n:50s} {(e - s) / 1e3:6.1f} gap {gap:6.1f} grid {k['Grid_Size_X']:>8s} {api.get(k['Correlation_Id'], '?')}")
print(f"busy {busy:.1f} us, idle gaps {gaps:.1f} us, {b - a} kernels")
