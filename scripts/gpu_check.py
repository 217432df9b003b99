"""First GPU-vs-oracle check (ad hoc; the pytest versions live in tests/)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle.oracle import Oracle  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from pychemkin_amd.mechanism import Mechanism  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
m = Mechanism.from_files(os.path.join(ROOT, "data/grimech30_chem.inp"), os.path.join(ROOT, "data/grimech30_thermo.dat"))
o = Oracle(m)
dm = _native.DeviceMechanism(m.to_tables())
KK = m.KK
print("device", torch.cuda.get_device_name(0), flush=True)

# ---- ROP
rng = np.random.default_rng(0)
n = 4096
T = rng.uniform(300, 3000, n)
P = 1.01325e6 * 10 ** rng.uniform(-1, 2, n)
Y = rng.dirichlet(0.5 * np.ones(KK), n).T.copy()
t0 = time.time()
w, cp, h = dm.rop_thermo(T, P, Y)
torch.cuda.synchronize()
print("rop kernel first call", time.time() - t0, flush=True)
w = w.cpu().numpy(); cp = cp.cpu().numpy(); h = h.cpu().numpy()
wo, cpo, ho = o.rop_batch(T, P, Y)
scale = np.max(np.abs(wo), axis=0, keepdims=True) + 1e-300
print("wdot max rel err (vs per-state max)", np.max(np.abs(w - wo) / scale), flush=True)
print("cp max rel err", np.max(np.abs(cp / cpo - 1)), "h max abs rel", np.max(np.abs(h - ho) / np.abs(ho).max()), flush=True)

# ---- reactors
def mix(phi):
    X = np.zeros(KK); alpha = 2 / 0.21
    X[13] = phi; X[3] = 0.21 * alpha; X[47] = 0.79 * alpha; X /= X.sum()
    return X * m.wt / (X * m.wt).sum()

cases = [(1200, 1, 1.0, 1), (1200, 1, 1.0, 2), (1100, 1, 0.5, 1), (1700, 100, 2.0, 1), (1000, 3, 0.7, 2), (1400, 10, 1.0, 1)]
T0 = np.array([c[0] for c in cases], float)
P0 = np.array([c[1] for c in cases], float) * 1.01325e6
Y0 = np.stack([mix(c[2]) for c in cases])
prob = np.array([c[3] for c in cases], np.int32)
cfg = _native.make_cfg(energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
t0 = time.time()
res = dm.reactor_run(cfg, prob, T0, P0, np.ones(len(cases)), Y0)
torch.cuda.synchronize()
print("reactor kernel", time.time() - t0, flush=True)
st = res["stats"].cpu().numpy()
for i, c in enumerate(cases):
    r, Ye = o.reactor(c[0], c[1] * 1.01325e6, 1.0, Y0[i], problem=c[3], energy=1, t_end=1.0, atol=1e-10, rtol=1e-8,
                      ign_mode="TIFP")
    print(c, "GPU tau %.8e T %.6f st %s | CPU tau %.8e T %.6f nst %d nlu %d | dtau %.2e dT %.2e dY %.2e" % (
        res["tau"][i].item(), res["T"][i].item(), st[i].tolist(), r.tau, r.T, r.nst, r.nlu,
        abs(res["tau"][i].item() / r.tau - 1), abs(res["T"][i].item() / r.T - 1),
        np.max(np.abs(res["Y"][i].cpu().numpy() - Ye))), flush=True)
