"""Diagnostic: the bench's HCCI sweep on the GPU -- failing cylinders, their status and step counts,
and the oracle on the same cylinders (test infrastructure: the oracle is only the checker here)."""
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
from pychemkin_amd import transport as trn  # noqa: E402

m = bench.mechanism()
dev = torch.device("cuda", 0)
dm = _native.DeviceMechanism(m.to_tables(), device=dev)
T0, P0, Y0 = bench.model_sweep(m, 1, 0, 16 ** 3 * 4, 420.0, 520.0, bench.P_ATM, 2 * bench.P_ATM, 0.3, 1.0)
params = trn.species_params(trn.parse_transport_text(open(os.path.join(ROOT, "data", "grimech30_transport.dat")).read()),
                            m.species)
fits = np.hstack([trn.viscosity_fits(m.wt, params), trn.conductivity_fits(m.wt, params, m.to_tables()["thermo"])])
tran = torch.tensor(fits, dtype=torch.float64, device=dev)
run = dict(bench.RUN, t_end=258.0 / 6000.0, nneg="--nneg" in sys.argv)
cfg = _native.make_cfg(engine=bench.hcci_block(), tran=tran, **run)
res = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, np.full(len(T0), 4, np.int32), T0, P0, np.ones(len(T0)),
                                                      Y0).items()}
st = res["stats"]
bad = np.nonzero(st[:, 6] != 0)[0]
out = {"n": len(T0), "failed": bad.tolist(), "status": st[bad, 6].tolist(), "nst": st[bad, 0].tolist(),
       "nst_p50_p99_max": [float(np.percentile(st[:, 0], 50)), float(np.percentile(st[:, 0], 99)), int(st[:, 0].max())],
       "cases": [(float(T0[i]), float(P0[i])) for i in bad]}
from oracle.oracle import Oracle  # noqa: E402
from test_engine import tran_fits  # noqa: E402

orc = Oracle(m)
tf = tran_fits(m)
out["oracle"] = []
for i in bad[:5]:
    r, _ = orc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=4, engine=bench.hcci_block(), tran=tf, **run)
    out["oracle"].append({"i": int(i), "status": r.status, "nst": r.nst, "tau": r.tau, "gpu_tau": float(res["tau"][i]),
                          "gpu_T": float(res["T"][i]), "T": r.T})
print(json.dumps(out))
