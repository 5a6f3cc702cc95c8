"""HIP API calls and kernel launches per adaptive step from a rocprofv3
--kernel-trace --hip-runtime-trace run of tools/adapt_loop.py: steps are
delimited by the launches of the check_for_adaptation kernel (k_adapt_diff).
usage: python tools/api_census.py <rocprof dir> [first step] [last step]"""
import collections
import csv
import sys

d = sys.argv[1]
tr = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
kt = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
marks = sorted(int(r["Start_Timestamp"]) for r in tr if False)
starts = sorted(int(k["Start_Timestamp"]) for k in kt if ("k_adapt_diff" in k["Kernel_Name"] or "k_adapt_faces" in k["Kernel_Name"]))
# the API call that launched each k_adapt_diff (by correlation id) marks a step
launch_of = {r["Correlation_Id"]: int(r["Start_Timestamp"]) for r in tr}
bounds = sorted(launch_of[k["Correlation_Id"]] for k in kt if ("k_adapt_diff" in k["Kernel_Name"] or "k_adapt_faces" in k["Kernel_Name"])
                and k["Correlation_Id"] in launch_of)
a = int(sys.argv[2]) if len(sys.argv) > 2 else len(bounds) - 9
b = int(sys.argv[3]) if len(sys.argv) > 3 else len(bounds) - 1
lo, hi = bounds[a], bounds[b]
steps = b - a
calls, dur = collections.Counter(), collections.Counter()
for r in tr:
    t = int(r["Start_Timestamp"])
    if lo <= t < hi:
        calls[r["Function"]] += 1
        dur[r["Function"]] += int(r["End_Timestamp"]) - t
print(f"steps {a}..{b} ({steps}): wall {(hi - lo) / 1e6 / steps:.2f} ms/step, "
      f"API time {sum(dur.values()) / 1e6 / steps:.2f} ms/step, {sum(calls.values()) / steps:.0f} calls/step")
for f, n in calls.most_common(14):
    print(f"  {f:32s} {n / steps:7.1f}/step  {dur[f] / 1e3 / steps:8.1f} us/step  avg {dur[f] / n / 1e3:6.1f} us")
kc, kd = collections.Counter(), collections.Counter()
for k in kt:
    t = int(k["Start_Timestamp"])
    if lo <= t < hi:
        name = k["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        kc[name] += 1
        kd[name] += int(k["End_Timestamp"]) - t
print(f"kernels: {sum(kc.values()) / steps:.0f} launches/step, {sum(kd.values()) / 1e6 / steps:.3f} ms/step busy")
for f, n in kd.most_common(int(sys.argv[4]) if len(sys.argv) > 4 else 40):
    print(f"  {f:60s} {kc[f] / steps:5.1f}/step {n / 1e3 / steps:8.1f} us/step  avg {n / 1e3 / kc[f]:6.1f} us")
