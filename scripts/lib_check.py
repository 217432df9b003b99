"""Quick GPU sanity check of libckmi variants: a few bench reactors against the oracle.

    python scripts/lib_check.py lib1.so [lib2.so ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json, numpy as np
sys.path.insert(0, %r)
import torch, bench
from pychemkin_amd import _native
from oracle.oracle import Oracle
mech = bench.mechanism()
dm = _native.DeviceMechanism(mech.to_tables(), device=0)
T0, P0, Y0, _ = bench.sweep(mech, 1, 0)
idx = np.arange(0, len(T0), len(T0) // 16)[:16]
res = dm.reactor_run(_native.make_cfg(**bench.RUN), np.ones(len(idx), np.int32), T0[idx], P0[idx], np.ones(len(idx)),
                     Y0[idx])
st = res["stats"].cpu().numpy()
o = Oracle(mech)
errs = []
for i in range(4):
    r, _ = o.reactor(T0[idx[i]], P0[idx[i]], 1.0, Y0[idx[i]], problem=1, **bench.RUN)
    errs.append(abs(res["tau"][i].item() / r.tau - 1))
print(json.dumps({"status": st[:, 6].tolist(), "steps": st[:, 0].tolist()[:6], "tau_rel_err": errs}))
"""
for lib in sys.argv[1:]:
    env = dict(os.environ, CKMI_LIB=os.path.abspath(lib))
    r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=300)
    print(os.path.basename(lib), r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-1500:], flush=True)
