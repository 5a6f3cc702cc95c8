"""Summarise a rocprofv3 run of bench.py into profiles/<tag>_summary.json.

Inputs (from tools/gpu_r1f.sh): <dir>/trace/run_kernel_stats.csv (kernel
trace + stats), <dir>/fetch/run_counter_collection.csv (--pmc FETCH_SIZE) and
<dir>/write/run_counter_collection.csv (--pmc WRITE_SIZE), each a separate
pass.  HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.
"""
import csv
import json
import statistics
import sys

KERNEL = "k_gol26v"


def headline_launches(prof_dir, n):
    """Durations (ns) of the bench's headline launches: the first n launches of
    the stencil kernel at its full grid size, in dispatch order (bench.py runs
    the headline loop before the secondary configs, whose RCCL-halo line
    launches the same kernel over the inner and outer slices)."""
    rows = [r for r in csv.DictReader(open(f"{prof_dir}/trace/run_kernel_trace.csv")) if KERNEL in r["Kernel_Name"]]
    full = max(int(r["Grid_Size_X"]) for r in rows)
    rows = sorted((r for r in rows if int(r["Grid_Size_X"]) == full), key=lambda r: int(r["Start_Timestamp"]))[:n]
    return rows[0]["Kernel_Name"], [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]


def main(prof_dir, tag, cells_per_launch, headline_n=0):
    stats = list(csv.DictReader(open(f"{prof_dir}/trace/run_kernel_stats.csv")))
    k = [r for r in stats if KERNEL in r["Name"]][0]
    if headline_n:
        name, durs = headline_launches(prof_dir, headline_n)
        k = {"Name": name, "Calls": len(durs), "AverageNs": statistics.mean(durs)}
    fetch = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{prof_dir}/fetch/run_counter_collection.csv"))
             if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    write = [float(r["Counter_Value"]) for r in csv.DictReader(open(f"{prof_dir}/write/run_counter_collection.csv"))
             if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
    fetch_b = 2 * statistics.median(fetch) * 1024
    write_b = statistics.median(write) * 1024
    alg = 12 * cells_per_launch
    avg_ns = float(k["AverageNs"])
    out = {
        "kernel": k["Name"],
        "calls": int(k["Calls"]),
        "average_ns": avg_ns,
        "cells_per_launch": cells_per_launch,
        "algorithmic_bytes_per_launch": alg,
        "achieved_GBs": alg / avg_ns,
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": fetch_b + write_b,
        "traffic_over_algorithmic": (fetch_b + write_b) / alg,
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes; separate --pmc passes",
    }
    json.dump(out, open(f"profiles/{tag}_summary.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2048 ** 3,
         int(sys.argv[4]) if len(sys.argv) > 4 else 0)
