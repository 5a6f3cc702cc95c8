"""Device idle gaps of a rocprofv3 kernel + HIP-runtime trace of tools/adapt_loop.py (steps marked by
k_adapt_diff): per-step wall and kernel-busy time, and the idle time split by the runtime call in flight
(none: host work).  usage: python3 tools/idle_gaps.py <rocprof output dir>"""
import csv, sys, collections
d = sys.argv[1]
K = [r for r in csv.DictReader(open(d + "/run_kernel_trace.csv"))]
A = [r for r in csv.DictReader(open(d + "/run_hip_api_trace.csv"))]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in K)
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in A)
# steps: find k_adapt_diff launches (one per check_for_adaptation) as step markers
marks = [s for s, e, n in ks if "k_adapt_diff" in n]
print("steps", len(marks))
i0, i1 = len(marks) - 6, len(marks) - 2
t0, t1 = marks[i0], marks[i1]
nsteps = i1 - i0
# union of kernel busy intervals
busy = 0
gaps = []
last = t0
for s, e, n in ks:
    if e < t0 or s > t1: continue
    s, e = max(s, t0), min(e, t1)
    if s > last:
        gaps.append((last, s))
    busy += max(0, e - max(s, last))
    last = max(last, e)
wall = t1 - t0
print(f"per step wall {wall/nsteps/1e3:.2f} us? -> {wall/nsteps/1e6:.3f} ms, busy {busy/nsteps/1e6:.3f} ms")
# classify gaps > 20 us by the API calls overlapping them
cls = collections.Counter()
tot = 0
for g0, g1 in gaps:
    L = g1 - g0
    if L < 20000: continue
    tot += L
    # API time inside the gap
    inside = collections.Counter()
    for s, e, f in api:
        if e < g0 or s > g1: continue
        inside[f] += min(e, g1) - max(s, g0)
    apit = sum(inside.values())
    top = inside.most_common(1)[0][0] if inside else "-"
    cls["api:" + top] += min(apit, L)
    cls["host(no api)"] += max(0, L - apit)
print(f"gaps >20us per step: {tot/nsteps/1e6:.3f} ms")
for k, v in cls.most_common(12):
    print(f"  {k:40s} {v/nsteps/1e6:.3f} ms/step")
# one step: gaps > 100 us with neighbors
import bisect
apis = [a[0] for a in api]
print("\nlargest gaps of step", i1 - 1)
s0, s1 = marks[i1 - 1], marks[i1]
G = [(g1 - g0, g0, g1) for g0, g1 in gaps if g0 >= s0 and g1 <= s1 and g1 - g0 > 100000]
for L, g0, g1 in sorted(G, reverse=True)[:14]:
    j = bisect.bisect_left(apis, g0)
    before = [api[x][2] for x in range(max(0, j - 2), j)]
    k = bisect.bisect_left(apis, g1)
    after = [api[x][2] for x in range(k - 1, min(len(api), k + 1))]
    kb = [n for s, e, n in ks if e <= g0][-1:]
    ka = [n for s, e, n in ks if s >= g1][:1]
    print(f"{L/1e3:8.0f} us at +{(g0-s0)/1e3:7.0f}  after kernel {kb} before kernel {ka}; api before {before} after {after}")
