"""Per-launch HBM bytes of the reactor and ROP kernels from scripts/pmc_traffic.sh output.

FETCH_SIZE (KiB) is doubled per the gfx950 calibration (MI355X_MICROARCH.md, HBM section: it
tallies 128-B requests at 64 B); WRITE_SIZE (KiB) is taken as is.  Output: profiles/traffic.json
format, {"reactor": {...}, "rop": {...}}, averaged over the dispatches of each kernel.
"""
import collections
import csv
import re
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            kind = ("reactor" if "reactor_kernel" in k else
                    "rop" if re.search(r"rop_kernel<0, 1[,>]", k) else        # GRI-3.0 (KK <= 63)
                    "rop_161sp" if re.search(r"rop_kernel<0, 3[,>]", k) else  # synthetic 161-species mechanism
                    "lu" if "lu_factor_kernel" in k else None)
            if kind is None:
                continue
            per[(kind, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (kind, _, cname), v in per.items():
            acc[kind][cname].append(v)
    out = {}
    for kind, c in acc.items():
        fetch = 2.0 * 1024 * sum(c["FETCH_SIZE"]) / max(len(c["FETCH_SIZE"]), 1)
        write = 1024 * sum(c["WRITE_SIZE"]) / max(len(c["WRITE_SIZE"]), 1)
        out[kind] = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                     "dispatches": len(c["FETCH_SIZE"])}
    # units per launch of the bench workload (bench.py defaults)
    if "reactor" in out:
        out["reactor"]["units"] = 65536
    if "rop" in out:
        out["rop"]["units"] = 10_000_000
    if "rop_161sp" in out:
        out["rop_161sp"]["units"] = 1_000_000
    if "lu" in out:
        out["lu"]["units"] = 16384
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
