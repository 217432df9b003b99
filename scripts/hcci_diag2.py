"""Diagnostic: trajectory of one failing HCCI cylinder (GPU vs oracle)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from test_engine import tran_fits  # noqa: E402

m = bench.mechanism()
dev = torch.device("cuda", 0)
dm = _native.DeviceMechanism(m.to_tables(), device=dev)
T0, P0, Y0 = bench.model_sweep(m, 1, 0, 16 ** 3 * 4, 420.0, 520.0, bench.P_ATM, 2 * bench.P_ATM, 0.3, 1.0)
tf = tran_fits(m)
tran = torch.tensor(tf, dtype=torch.float64, device=dev)
out = {}
for mode in ("ht", "adiabatic"):
    e = bench.hcci_block()
    if mode == "adiabatic":
        e[7] = 0.0
    run = dict(bench.RUN, t_end=258.0 / 6000.0)
    ts = np.linspace(0.0, run["t_end"], 87)
    idx = [378, 389, 1738]
    cfg = _native.make_cfg(engine=e, tran=tran if mode == "ht" else None, **run)
    res = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, np.full(3, 4, np.int32), T0[idx], P0[idx], np.ones(3),
                                                          Y0[idx], t_save=ts).items()}
    orc = Oracle(m)
    for j, i in enumerate(idx):
        r, _, (_, ys, ps, vs) = orc.reactor(T0[i], P0[i], 1.0, Y0[i], t_save=ts, problem=4, engine=e,
                                            tran=tf if mode == "ht" else None, **run)
        g = res["y_save"][j][:, 0]
        out[f"{mode}_{i}"] = {"gpu_status": int(res["stats"][j, 6]), "gpu_nst": int(res["stats"][j, 0]),
                              "gpu_stats": res["stats"][j].tolist(),
                              "oracle_stats": [r.nst, r.nfe, r.nje, r.nlu, r.ncf, r.nef],
                              "oracle_nst": r.nst, "T_gpu": np.round(g, 2).tolist(), "T_oracle": np.round(ys[:, 0], 2).tolist()}
print(json.dumps(out))
