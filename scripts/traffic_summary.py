"""Per-launch HBM bytes of the reactor and ROP kernels from scripts/pmc_traffic.sh output.

    python scripts/traffic_summary.py gpurun_out/traffic_TAG [--line c4|c5|pfr|hcci|ropext]
      (a run of that bench line only: its kernel's largest dispatch is the line's launch -- the smaller
      ones are the line's warm-up and the tiny headline run that always precedes it; ropext: the
      161-species ROP dispatches of that run are the extended-mechanism line's, keyed rop_ext[_jit])

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
    line = sys.argv[sys.argv.index("--line") + 1] if "--line" in sys.argv else ("c4" if "--c4" in sys.argv else "c3")
    # reactor_kernel dispatches of a run belong to one line: c3 (default) or c4
    reactor_key = "reactor_c4" if line == "c4" else "reactor"
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            kind = ("big_reactor" if "big_reactor_kernel" in k else            # configs[4] (c5 line)
                    # the FP64-inverse companion launch that runs (here: skips) the plug-flow reactors
                    reactor_key + "_pfr_launch" if re.search(r"(^|[^_])reactor_kernel<\d+, (true|false), true>", k) else
                    reactor_key if re.search(r"(^|[^_])reactor_kernel", k) else  # configs[2] / [3] (c3 / c4)
                    "rop" if re.search(r"rop_kernel<0, 1[,>]", k) else        # GRI-3.0 (KK <= 63), generic
                    "rop_161sp" if re.search(r"rop_kernel<0, 3[,>]", k) else  # synthetic 161-species, generic
                    "rop_jit" if "ckjit_rop_k53_" in k else                   # specialised kernels
                    "rop_161sp_jit" if "ckjit_rop_k161_" in k else
                    "lu" if "lu_factor_kernel" in k else None)
            if kind is None:
                continue
            per[(kind, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (kind, _, cname), v in per.items():
            if line == "ropext":  # that run's other kernels are its tiny headline run: not the lines' launches
                if not kind.startswith("rop_161sp"):
                    continue
                kind = "rop_ext" + kind[len("rop_161sp"):]
            acc[kind][cname].append(v)
    out = {}
    # the line's own kernel and its key in profiles/traffic.json (largest dispatch only)
    single = {"c4": ("reactor_c4", "reactor_c4"), "c5": ("big_reactor", "big_reactor_c5"),
              "pfr": ("reactor_pfr_launch", "reactor_pfr"), "hcci": ("reactor_pfr_launch", "reactor_hcci")}.get(line)
    if single is not None:
        c = acc[single[0]]
        fetch = 2.0 * 1024 * max(c["FETCH_SIZE"])
        write = 1024 * max(c["WRITE_SIZE"])
        units = {"c4": 2 ** 20, "c5": 262144, "pfr": 16 ** 3, "hcci": 25 ** 3}[line]  # bench.py model_line totals
        out[single[1]] = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                          "dispatches": 1, "units": units}
        print(json.dumps(out, indent=1))
        return
    for kind, c in acc.items():
        if kind.startswith("reactor_c4"):  # the c4 run's tiny headline dispatches are dropped: largest dispatch only
            fetch = 2.0 * 1024 * max(c["FETCH_SIZE"])
            write = 1024 * max(c["WRITE_SIZE"])
            out[kind] = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write, "dispatches": 1}
            continue
        fetch = 2.0 * 1024 * sum(c["FETCH_SIZE"]) / max(len(c["FETCH_SIZE"]), 1)
        write = 1024 * sum(c["WRITE_SIZE"]) / max(len(c["WRITE_SIZE"]), 1)
        out[kind] = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                     "dispatches": len(c["FETCH_SIZE"])}
    # units per launch of the bench workload (bench.py defaults)
    units = {"reactor": 65536, "reactor_c4": 2 ** 20, "big_reactor": 262144, "rop": 10_000_000, "rop_jit": 10_000_000,
             "rop_161sp": 1_000_000, "rop_161sp_jit": 1_000_000, "rop_ext": 1_000_000, "rop_ext_jit": 1_000_000}
    for k, u in units.items():
        if k in out:
            out[k]["units"] = u
    if "lu" in out:
        out["lu"]["units"] = 16384
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
