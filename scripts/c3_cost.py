"""Per-reactor solver statistics of the c3 sweep (configs[2]) for a work-queue / tail analysis: writes
gpurun_out/c3_cost.npz (stats, T0, P0) and prints the step-count spread."""
import sys, os, json, numpy as np
sys.path.insert(0, os.getcwd())
import torch, bench
from pychemkin_amd import _native
mech = bench.mechanism()
dm = _native.DeviceMechanism(mech.to_tables(), device=0)
T0, P0, Y0, prob = bench.sweep(mech, 1, 0)
cfg = _native.make_cfg(**bench.RUN)
args = (prob, T0, P0, np.ones(len(T0)), Y0)
dm.reactor_run(cfg, *args); torch.cuda.synchronize()
res = dm.reactor_run(cfg, *args); torch.cuda.synchronize()
st = res["stats"].cpu().numpy()
np.savez("gpurun_out/c3_cost.npz", st=st, T0=T0, P0=P0)
nst, nfe = st[:, 0].astype(float), st[:, 1].astype(float)
print(json.dumps({"n": len(T0), "nst_mean": nst.mean(), "nst_max": nst.max(), "nst_p99": float(np.percentile(nst, 99)),
                  "nfe_mean": nfe.mean(), "nfe_max": nfe.max()}))
