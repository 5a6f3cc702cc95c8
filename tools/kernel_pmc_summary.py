"""Per-kernel HBM traffic of a program from three rocprofv3 runs of it:
<dir>/trace (--kernel-trace --stats), <dir>/fetch (--pmc FETCH_SIZE) and
<dir>/write (--pmc WRITE_SIZE), each a separate pass (MI355X_MICROARCH.md
HBM section: FETCH_SIZE and WRITE_SIZE in KiB; on gfx950 FETCH_SIZE reports
half of a wide coalesced read, so it is doubled).
usage: python tools/kernel_pmc_summary.py <dir> <out.json> [name substrings...]"""
import collections
import csv
import json
import statistics
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("dccrgx::", "")


def main(d, out, keys):
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = {}
    for which, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f"{d}/{which}/run_counter_collection.csv")):
            if r["Counter_Name"] == counter:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
        cnt[which] = vals
    res = {}
    for k, v in dur.items():
        if keys and not any(s in k for s in keys):
            continue
        f = cnt["fetch"].get(k, [])
        w = cnt["write"].get(k, [])
        res[k] = {"calls": len(v), "average_ns": statistics.mean(v),
                  "fetch_bytes": 2 * statistics.mean(f) if f else None,
                  "write_bytes": statistics.mean(w) if w else None}
    json.dump({"note": "per launch; FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes; separate --pmc passes",
               "kernels": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
