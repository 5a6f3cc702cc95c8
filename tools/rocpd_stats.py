"""Kernel statistics from a rocprofv3 results database (rocpd SQLite, the
default output of rocprofv3 --kernel-trace here): per kernel name the
number of dispatches, total / average / min / max duration in ns, as the
*_kernel_stats.csv of the CSV output.  usage: rocpd_stats.py results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": r[3], "Percentage": 100.0 * r[2] / tot,
             "MinNs": r[4], "MaxNs": r[5]} for r in rows]


if __name__ == "__main__":
    out = stats(sys.argv[1])
    w = csv.DictWriter(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout, fieldnames=list(out[0]))
    w.writeheader()
    w.writerows(out)
