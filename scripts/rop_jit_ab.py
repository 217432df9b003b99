"""A/B of generator settings of the specialised ROP kernel (one child process per setting).

    python scripts/rop_jit_ab.py CKMI_JIT_GROUP=1 CKMI_JIT_GROUP=4 ... [--n 10000000]

Each child builds the bench's random (T, P, Y) states, compiles the kernel with the given
environment, checks it against the generic kernel and reports the HIP-event time per launch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, json, time, numpy as np
sys.path.insert(0, %r)
import torch, bench
from pychemkin_amd import _native
ns = %d
mech = bench.mechanism()
dm = _native.DeviceMechanism(mech.to_tables(), device=0)
rng = np.random.default_rng(0)
dev = "cuda:0"
Ts = torch.as_tensor(rng.uniform(300.0, 3000.0, ns), device=dev)
Ps = torch.as_tensor(bench.P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, ns), device=dev)
Ys = torch.as_tensor(rng.dirichlet(0.5 * np.ones(mech.KK), ns).T.copy(), device=dev)
out = [torch.empty((mech.KK, ns), dtype=torch.float64, device=dev), torch.empty(ns, dtype=torch.float64, device=dev),
       torch.empty(ns, dtype=torch.float64, device=dev)]
_native.set_rop_path(1)
dm.rop_thermo(Ts, Ps, Ys, *out); torch.cuda.synchronize()
ref = out[0][:, :100000].cpu().numpy()
_native.set_rop_path(2)
t0 = time.time(); dm.rop_thermo(Ts, Ps, Ys, *out); torch.cuda.synchronize(); tc = time.time() - t0
got = out[0][:, :100000].cpu().numpy()
err = float(np.max(np.abs(got - ref) / np.max(np.abs(ref), axis=0, keepdims=True)))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5): dm.rop_thermo(Ts, Ps, Ys, *out)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(json.dumps({"ms": ms, "states_per_s": ns / ms * 1e3, "compile_s": tc, "max_rel_vs_generic": err}))
"""


def main():
    sets = [a for a in sys.argv[1:] if "=" in a and not a.startswith("--")]
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 10_000_000
    res = {}
    for st in sets:
        env = dict(os.environ)
        for kv in st.split(","):
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, n)], env=env, capture_output=True, text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        res[st] = json.loads(line[-1]) if line else {"error": r.stderr[-2000:]}
        print(st, res[st], flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
