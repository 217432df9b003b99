"""Render a rocprofv3 --stats kernel summary (CSV) plus the bench JSON of the same run as markdown.

    python scripts/stats_md.py TITLE gpurun_out/prof_TAG/run_kernel_stats.csv gpurun_out/bench_prof_TAG.json \
        [notes...] > profiles/TAG_kernel_stats.md
"""
import csv
import json
import sys


def main():
    title, stats, bench = sys.argv[1:4]
    notes = sys.argv[4:]
    rows = list(csv.DictReader(open(stats)))
    print(f"# {title}\n")
    for n in notes:
        print(n + "\n")
    b = None
    for line in open(bench):
        if line.startswith("{"):
            b = json.loads(line)
    if b:
        print(f"bench.py in-process HIP-event kernel time for the same run: {b['roofline']['kernel_ms']:.1f} ms/launch "
              f"(reactor), {b['rop']['ms_per_launch']:.2f} ms/launch (ROP).\n")
    print("| kernel | calls | total ms | avg ms | min ms | max ms | share |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e6:.3f} | {float(r['MinNs']) / 1e6:.3f} | {float(r['MaxNs']) / 1e6:.3f} | "
              f"{float(r['Percentage']):.1f}% |")
    if b:
        print("\n```json\n" + json.dumps(b) + "\n```")


if __name__ == "__main__":
    main()
