"""Summarise kernel dispatches of a rocprofv3 rocpd database (or a *_kernel_stats.csv) per kernel.

Usage: python scripts/rocpd_stats.py <results.db | kernel_stats.csv> [> profiles/<name>.md]
Prints a markdown table: kernel, calls, total ms, average ms, min ms, max ms, share.
"""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name} order by sum(end-start) desc").fetchall()
    return [(r[0], int(r[1]), r[2] / 1e6, r[3] / 1e6, r[4] / 1e6, r[5] / 1e6) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6,
                        float(r["MinNs"]) / 1e6, float(r["MaxNs"]) / 1e6))
    return out


def main():
    p = sys.argv[1]
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    tot = sum(r[2] for r in rows) or 1.0
    print("| kernel | calls | total ms | avg ms | min ms | max ms | share |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        nm = r[0] if len(r[0]) < 90 else r[0][:87] + "..."
        print(f"| `{nm}` | {r[1]} | {r[2]:.3f} | {r[3]:.3f} | {r[4]:.3f} | {r[5]:.3f} | {100 * r[2] / tot:.1f}% |")


if __name__ == "__main__":
    main()
