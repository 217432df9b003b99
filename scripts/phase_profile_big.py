"""Per-phase cycle breakdown of the workgroup-per-reactor kernel (diagnostic build).

    python -c "from pychemkin_amd import build; build.build(prof=True)"
    CKMI_LIB=pychemkin_amd/_lib/libckmi_prof.so python scripts/phase_profile_big.py [n]

Runs n reactors of the configs[4] stand-in sweep (strided sample of bench.sweep_c5) and prints the
mean shader cycles per reactor in each phase, per call, and per integration step.
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = bench.big_mechanism()
    dm = _native.DeviceMechanism(m.to_tables(), device=0)
    T0, P0, Y0, prob = bench.sweep_c5(m, 1, 0)
    idx = np.arange(0, len(T0), max(1, len(T0) // n))[:n]
    buf = torch.zeros((len(idx), 16), dtype=torch.int64, device="cuda")
    L = _native.lib()
    L.ckmi_debug_big_phase_buffer.argtypes = [ct.c_void_p]
    assert L.ckmi_debug_big_phase_buffer(buf.data_ptr()) == 0
    res = dm.reactor_run(_native.make_cfg(**bench.RUN), prob[idx], T0[idx], P0[idx], np.ones(len(idx)), Y0[idx])
    torch.cuda.synchronize()
    st = res["stats"].cpu().numpy().astype(np.float64)
    ph = buf.cpu().numpy().astype(np.float64)
    names = ["rhs", "rhs_jac", "build", "factor", "solve", "total"]
    calls = {"rhs": st[:, 1] - st[:, 2], "rhs_jac": st[:, 2], "build": st[:, 3], "factor": st[:, 3],
             "solve": st[:, 7]}
    tot = ph[:, 5].sum()
    out = {"reactors": int(len(idx)), "mean_steps": float(st[:, 0].mean()), "phases": {}}
    for k, nm in enumerate(names):
        c = ph[:, k].sum()
        d = {"frac_of_total": c / tot, "cycles_per_step": c / st[:, 0].sum()}
        if nm in calls:
            d["cycles_per_call"] = c / max(calls[nm].sum(), 1)
            d["calls_per_step"] = calls[nm].sum() / st[:, 0].sum()
        out["phases"][nm] = d
    fac = ph[:, 3].sum()
    # wave 0's view of the factorisation (MFMA panels): own panels (pivot steps + publication), barrier
    # wait, own panels' entry + column transposition, pivot-row gather, B loads + MFMA update, owner column
    # restore (VALU build CKMI_BIG_VALU: search, publish, update)
    names_f = ["own_panel_steps", "barrier", "own_panel_entry", "pivot_row_gather", "mfma_update", "restore"]
    out["factor_split"] = {nm: ph[:, 6 + k].sum() / fac for k, nm in enumerate(names_f) }
    npan = max(calls["factor"].sum(), 1) * ((m.KK + 1 + 3) // 4)
    out["factor_split"]["cycles_per_panel"] = {nm: ph[:, 6 + k].sum() / npan for k, nm in enumerate(names_f) }
    other = tot - ph[:, :5].sum()
    out["phases"]["control"] = {"frac_of_total": other / tot, "cycles_per_step": other / st[:, 0].sum()}
    # the control states' own time (state-machine passes; the Newton iteration's solve and the setup's
    # build + factorisation are subtracted / excluded)
    nst = st[:, 0].sum()
    newton = ph[:, 12].sum() - ph[:, 4].sum()
    out["control_split_cycles_per_step"] = {
        "newton_iter_excl_solve": newton / nst, "step_complete": ph[:, 13].sum() / nst,
        "step_begin_end": ph[:, 14].sum() / nst, "other_states": ph[:, 15].sum() / nst,
        "unattributed": (other - newton - ph[:, 13:16].sum()) / nst}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
