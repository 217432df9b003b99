"""Diagnostic: which part of the engine heat transfer makes the failing cylinders fail on the GPU."""
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
from test_engine import tran_fits  # noqa: E402

m = bench.mechanism()
dev = torch.device("cuda", 0)
dm = _native.DeviceMechanism(m.to_tables(), device=dev)
T0, P0, Y0 = bench.model_sweep(m, 1, 0, 16 ** 3 * 4, 420.0, 520.0, bench.P_ATM, 2 * bench.P_ATM, 0.3, 1.0)
tran = torch.tensor(tran_fits(m), dtype=torch.float64, device=dev)
idx = [378, 389, 1738]
out = {}
variants = {"base": {}, "a_tiny": {8: 1e-9}, "b0": {9: 0.0}, "C2_0": {14: 0.0}, "Twall_600": {11: 600.0}}
for name, mods in variants.items():
    for extra in ({}, {"nneg": True}, {"rtol": 1e-10, "atol": 1e-14}):
        e = bench.hcci_block()
        for k, v in mods.items():
            e[k] = v
        run = dict(bench.RUN, t_end=258.0 / 6000.0)
        run.update(extra)
        cfg = _native.make_cfg(engine=e, tran=tran, **run)
        res = dm.reactor_run(cfg, np.full(3, 4, np.int32), T0[idx], P0[idx], np.ones(3), Y0[idx])
        st = res["stats"].cpu().numpy()
        out[name + "_" + "_".join(f"{k}{v}" for k, v in extra.items())] = [[int(x) for x in st[j, [0, 4, 5, 6]]] for j in range(3)]
print(json.dumps(out))
