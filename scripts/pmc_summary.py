"""Summarise rocprofv3 --pmc CSV passes (scripts/pmc_passes.sh) per kernel: counter totals
summed over dimensions, one row per kernel name (dispatches summed).

    python scripts/pmc_summary.py gpurun_out/pmc_TAG [--json]
"""
import collections
import csv
import glob
import json
import os
import sys


def load(root):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            short = ("big_reactor" if "big_reactor_kernel" in k else "reactor" if "reactor_kernel" in k else
                     "rop_jit" if "ckjit_rop" in k else "rop" if "rop_kernel" in k else k[:40])
            tot[short][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[short].add((f, row["Dispatch_Id"]))
    return tot, disp


def main():
    root = sys.argv[1]
    tot, disp = load(root)
    out = {}
    for k in ("reactor", "big_reactor", "rop", "rop_jit"):
        if k not in tot:
            continue
        c = tot[k]
        d = dict(c)
        # SQ_*_CYCLES / WAIT / ACTIVE are in quad-cycles on CDNA (MI355X_MICROARCH.md constants table)
        if c.get("SQ_WAVE_CYCLES"):
            d["valu_active_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_ACTIVE_INST_VALU") else None
            d["wait_inst_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
        f64 = c.get("SQ_INSTS_VALU_FMA_F64", 0) * 2 + c.get("SQ_INSTS_VALU_MUL_F64", 0) + c.get("SQ_INSTS_VALU_ADD_F64", 0)
        d["fp64_flops_counted"] = f64 * 64
        if "SQ_INSTS_VALU_MFMA_F64" in c:  # every f64 MFMA here is 16x16x4: 1024 FMA = 2048 FLOP per wave instr
            d["mfma_f64_flops_from_insts"] = c["SQ_INSTS_VALU_MFMA_F64"] * 2048
        if "FETCH_SIZE" in c:
            d["fetch_bytes_x2_calibrated"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            d["write_bytes"] = c["WRITE_SIZE"] * 1024
        out[k] = d
    if "--json" in sys.argv:
        print(json.dumps(out, indent=1))
    else:
        for k, d in out.items():
            print(f"== {k}")
            for n, v in sorted(d.items()):
                print(f"  {n:40s} {v:.6g}" if isinstance(v, float) else f"  {n:40s} {v}")


if __name__ == "__main__":
    main()
