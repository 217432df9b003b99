"""Element-drift diagnostic: GPU reactor kernel vs the oracle on the same configs[2] reactors.

Prints the distribution of the relative element drift |E y_end - E y_0| / max(E y_0) for a random
1024-reactor sample, then, for the 4 worst GPU reactors, the drift along a 41-point save grid on
both sides (where along the trajectory the GPU departs)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from conftest import CHEM, THERM  # noqa: E402

import bench  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from pychemkin_amd.mechanism import Mechanism  # noqa: E402


def drift(m, Y0, Y):
    ncf = m.ncf.astype(float)
    e0 = (Y0 / m.wt) @ ncf.T
    e1 = (Y / m.wt) @ ncf.T
    return np.max(np.abs(e1 - e0) / np.max(e0, axis=-1, keepdims=True), axis=-1)


m = Mechanism.from_files(CHEM, THERM)
o = Oracle(m)
dm = _native.DeviceMechanism(m.to_tables())
T0, P0, Y0, prob = bench.sweep(m, 1, 0)
idx = np.sort(np.random.default_rng(0).choice(T0.size, 1024, replace=False))
res = dm.reactor_run(_native.make_cfg(**bench.RUN), prob[idx], T0[idx], P0[idx], np.ones(idx.size), Y0[idx])
dg = drift(m, Y0[idx], res["Y"].cpu().numpy())
nf, _, Yo = o.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(idx.size), nthreads=16, **bench.RUN)
do = drift(m, Y0[idx], np.asarray(Yo))
q = [50, 90, 99, 100]
print("gpu drift pct", dict(zip(q, np.percentile(dg, q))))
print("orc drift pct", dict(zip(q, np.percentile(do, q))))
print("corr", np.corrcoef(np.log10(dg + 1e-18), np.log10(do + 1e-18))[0, 1])
w = np.argsort(dg)[-4:]
ts = np.linspace(0.0, 1.0, 201)
ts_d = ts.copy()
for j in w:
    i = idx[j]
    r = dm.reactor_run(_native.make_cfg(**bench.RUN), prob[i:i + 1], T0[i:i + 1], P0[i:i + 1], np.ones(1), Y0[i:i + 1],
                       t_save=ts_d)
    yg = r["y_save"][0].cpu().numpy()[:, 1:]
    st = r["stats"].cpu().numpy()[0]
    _, _, (_, yo, _, _) = o.reactor(T0[i], P0[i], 1.0, Y0[i], t_save=ts, problem=int(prob[i]), **bench.RUN)
    gg = drift(m, Y0[i][None, :], yg)
    oo = drift(m, Y0[i][None, :], yo[:, 1:])
    tau = r["tau"].cpu().numpy()[0]
    print(f"reactor {i}: T0 {T0[i]:.1f} P0 {P0[i]:.3e} tau {tau:.4e} stats {st.tolist()}")
    for k in range(0, ts.size, 10):
        print(f"   t {ts[k]:.3f}  gpu {gg[k]:.3e}  orc {oo[k]:.3e}")
