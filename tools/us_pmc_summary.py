"""Per-kernel counters of tools/user_stencil_bench.py (the staged and walk
launches of the game-of-life functor on 2048^3) from gpu_pass.sh's `us` and
`uspmc` steps: durations from <dir>/us_prof (--kernel-trace --stats), counters
from <dir>/uspmc_1..4 (one --pmc pass each: FETCH_SIZE, WRITE_SIZE, SQ_*,
TCC/TA/GRBM).  FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts
half of a wide coalesced read, so it is doubled (MI355X_MICROARCH.md).
usage: python tools/us_pmc_summary.py <dir> <out.json>"""
import collections
import csv
import glob
import json
import statistics
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("dccrgx::", "").replace("void ", "")


def kernel_key(name):
    s = short(name)
    return s.split("<")[0] if "<" in s else s


def main(d, out):
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{d}/us_prof/**/*kernel_trace.csv", recursive=True) + glob.glob(f"{d}/us_prof/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            dur[kernel_key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(set(glob.glob(f"{d}/uspmc_*/**/*counter_collection.csv", recursive=True) +
                        glob.glob(f"{d}/uspmc_*/*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k in sorted(set(dur) | set(vals)):
        if not any(s in k for s in ("k_staged", "k_user", "k_gol")):
            continue
        e = {}
        if dur.get(k):
            e["launches"] = len(dur[k])
            e["mean_us"] = statistics.mean(dur[k]) / 1e3
        for c, v in vals.get(k, {}).items():
            m = statistics.mean(v)
            if c == "FETCH_SIZE":
                e["fetch_bytes"] = 2 * m * 1024
            elif c == "WRITE_SIZE":
                e["write_bytes"] = m * 1024
            else:
                e[c] = m
        h, miss = e.get("TCC_HIT_sum"), e.get("TCC_MISS_sum")
        if h is not None and miss is not None and h + miss > 0:
            e["l2_hit_rate"] = h / (h + miss)
        if "mean_us" in e and "fetch_bytes" in e and "write_bytes" in e:
            e["hbm_GBps"] = (e["fetch_bytes"] + e["write_bytes"]) / (e["mean_us"] * 1e3)
        if e.get("SQ_BUSY_CYCLES") and e.get("SQ_WAIT_INST_ANY") is not None and e.get("SQ_WAVE_CYCLES"):
            e["wait_inst_frac"] = e["SQ_WAIT_INST_ANY"] / e["SQ_WAVE_CYCLES"]
        res[k] = e
    json.dump(res, open(out, "w"), indent=1)
    for k, e in res.items():
        print(k, json.dumps({a: (round(b, 4) if isinstance(b, float) else b) for a, b in e.items()}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
