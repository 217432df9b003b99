"""Wave-0 cycle split of lu_factor_kernel from a -DCKMI_LU_PHASE standalone build:
    python scripts/lu_phase.py lib_phase.so [lib_plain.so]
Phases (per matrix, summed over the 11 panels at n = 161): 0 load, 1 panel to LDS, 2 panel factor
(wave 0 alone; the register form splits it into 7 tile parking + panel load, 8 the 16 pivot
columns, 9 write-back + L11^-1, 10 the net permutation; 2 keeps the tile reload), 3 interchanges, 4 U12, 5 trailing
update, 6 store."""
import ctypes as ct
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lu_ab import time_lib  # noqa: E402

NAMES = ["load", "panel_to_lds", "panel_unpark", "interchange", "u12", "trailing", "store", "panel_park_load",
         "panel_columns", "panel_wb_l11inv", "panel_perm", "unused"]


def main():
    lib = ct.CDLL(sys.argv[1])
    out = (ct.c_ulonglong * 12)()
    nsys = 16384
    for newton in (False, True):
        lib.ckmi_lu_phase_get(out, 1)
        ms, *_ = time_lib(sys.argv[1], nsys=nsys, newton=newton, reps=2)
        lib.ckmi_lu_phase_get(out, 1)
        # reps=2: two launches; one workgroup-wave 0 per matrix
        per = [out[k] / (2 * nsys) for k in range(12)]
        tot = sum(per)
        print(json.dumps({"matrices": "newton" if newton else "randn", "ms": ms,
                          "cycles_per_matrix": {NAMES[k]: round(per[k]) for k in range(12)},
                          "frac": {NAMES[k]: round(per[k] / tot, 3) for k in range(12)}}), flush=True)
    for p in sys.argv[2:]:
        ms, *_ = time_lib(p, nsys=nsys)
        print(json.dumps({"lib": p, "ms": ms}), flush=True)


if __name__ == "__main__":
    main()
