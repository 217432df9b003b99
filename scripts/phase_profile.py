"""Per-phase cycle breakdown of the reactor kernel (diagnostic build, -DCKMI_PHASE_TIMERS).

    python pychemkin_amd/build.py --prof
    CKMI_LIB=pychemkin_amd/_lib/libckmi_prof.so python scripts/phase_profile.py [n]

Runs the bench workload's sweep (a strided subsample of n reactors) and prints, per reactor
mean, the shader cycles in RHS, Jacobian, LU factor, triangular solves and total, plus the
cycles per call of each.  s_memtime stamps cost ~10 % of wave time; compare phases, not wall.
"""
import ctypes as ct
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CKMI_LIB", os.path.join(ROOT, "pychemkin_amd", "_lib", "libckmi_prof.so"))
import torch  # noqa: E402

import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from pychemkin_amd.mechanism import Mechanism  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    mech = Mechanism.from_files(os.path.join(ROOT, "data", "grimech30_chem.inp"),
                                os.path.join(ROOT, "data", "grimech30_thermo.dat"))
    dm = _native.DeviceMechanism(mech.to_tables(), device=0)
    T0, P0, Y0, _ = bench.sweep(mech, 1, 0)
    prob, V0 = np.ones(len(T0), np.int32), np.ones(len(T0))
    idx = np.arange(0, len(T0), max(1, len(T0) // n))[:n]
    buf = torch.zeros((len(idx), 48), dtype=torch.int64, device="cuda:0")
    L = _native.lib()
    L.ckmi_debug_phase_buffer.argtypes = [ct.c_void_p]
    assert L.ckmi_debug_phase_buffer(buf.data_ptr()) == 0
    cfg = _native.make_cfg(**bench.RUN)
    res = dm.reactor_run(cfg, prob[idx], T0[idx], P0[idx], V0[idx], Y0[idx])
    torch.cuda.synchronize()
    ph = buf.cpu().numpy().astype(np.float64)
    st = res["stats"].cpu().numpy().astype(np.float64)
    names = ["rhs", "jac", "lu", "solve", "total"]
    counts = {"rhs": st[:, 1] - st[:, 2], "jac": st[:, 2], "lu": st[:, 3], "solve": st[:, 7]}
    out = {"reactors": int(len(idx)), "mean_steps": float(st[:, 0].mean())}
    for k, nm in enumerate(names):
        out[nm + "_cycles"] = float(ph[:, k].mean())
        if nm in counts:
            out[nm + "_cycles_per_call"] = float(ph[:, k].sum() / max(counts[nm].sum(), 1))
    for k, nm in zip((5, 6, 7), ("rhs_species_thirdbody", "rhs_reactions", "rhs_energy")):
        out[nm + "_cycles_per_call"] = float(ph[:, k].sum() / max(counts["rhs"].sum(), 1))
    states = ["NEXT", "START_F", "INITSTEP_F", "START_FINISH", "IGN0_F", "STEP_BEGIN", "STEP_ATTEMPT", "NLS_ATTEMPT",
              "NLS_F", "NLS_J", "SETUP", "NEWTON_ITER", "NEWTON_F", "NLS_FAIL", "STEP_CONVFAIL", "ERRTEST", "ERR_F",
              "STEP_COMPLETE", "STEP_END", "FINISH"]
    out["state_cycles_per_step"] = {nm: float(ph[:, 8 + k].mean() / out["mean_steps"]) for k, nm in enumerate(states)
                                    if ph[:, 8 + k].any()}
    out["newton_build_cycles_per_call"] = float(ph[:, 8 + 20].sum() / max(counts["lu"].sum(), 1))
    out["rhs_strip_cycles_per_call"] = [float(ph[:, 8 + 24 + k].sum() / max(counts["rhs"].sum(), 1)) for k in range(6)]
    acc = sum(out[nm + "_cycles"] for nm in names[:4])
    out["other_cycles"] = out["total_cycles"] - acc
    out["cycles_per_step"] = out["total_cycles"] / out["mean_steps"]
    for nm in names[:4] + ["other"]:
        out[nm + "_frac"] = out[nm + "_cycles"] / out["total_cycles"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
