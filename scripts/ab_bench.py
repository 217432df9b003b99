"""A/B timing of libckmi variants on the same GPU (alternating processes, same workload).

    python scripts/ab_bench.py pychemkin_amd/_lib/libA.so pychemkin_amd/_lib/libB.so [--reps 3] [--n 16384] [--rop | --c5]

Each rep runs every library in its own process (CKMI_LIB=...) on a strided subsample of the
bench sweep and reports the kernel time from HIP events; prints the per-library median.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, json, numpy as np
sys.path.insert(0, %r)
import ctypes, torch, bench
from pychemkin_amd import _native
# an older library of the same reactor ABI may lack later symbols: bind only what it exports
_L = ctypes.CDLL(_native.LIB_PATH)
for _k in [k for k in _native.PROTOTYPES if not hasattr(_L, k)]:
    _native.PROTOTYPES.pop(_k)
_native.ABI_VERSION = _L.ckmi_version()  # an A/B may time an older build of the same reactor entry points
n = %d
c5 = %r
mech = bench.big_mechanism() if c5 else bench.mechanism()
dm = _native.DeviceMechanism(mech.to_tables(), device=0)
T0, P0, Y0, prob = bench.sweep_c5(mech, 1, 0) if c5 else bench.sweep(mech, 1, 0)
idx = np.arange(0, len(T0), max(1, len(T0) // n))[:n]
args = (np.ones(len(idx), np.int32), T0[idx], P0[idx], np.ones(len(idx)), Y0[idx])
cfg = _native.make_cfg(**bench.RUN)
dm.reactor_run(cfg, *args); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); res = dm.reactor_run(cfg, *args); e1.record(); torch.cuda.synchronize()
st = res["stats"].cpu().numpy()
tau = res["tau"].cpu().numpy()
ref = os.environ.get("AB_TAU_REF")
d = {"ms": e0.elapsed_time(e1), "mean_stats": [round(float(x), 3) for x in st.mean(axis=0)],
     "fail": int((st[:, 6] != 0).sum()), "tau0": float(tau[0])}
if ref and os.path.exists(ref):
    t0 = np.load(ref)
    d["tau_max_rel_vs_ref"] = float(np.max(np.abs(tau - t0) / np.abs(t0)))
elif ref:
    np.save(ref, tau)
print(json.dumps(d))
"""

ROP_CHILD = r"""
import os, sys, json, numpy as np
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
wdot = torch.empty((mech.KK, ns), dtype=torch.float64, device=dev)
cp = torch.empty(ns, dtype=torch.float64, device=dev)
hh = torch.empty(ns, dtype=torch.float64, device=dev)
dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh)
e1.record(); torch.cuda.synchronize()
print(json.dumps({"ms": e0.elapsed_time(e1) / 3, "wsum": float(wdot[:, :1000].abs().sum().item())}))
"""


def main():
    # a library argument may carry environment settings for its runs: lib.so@CKMI_JIT_ORDER=0@CKMI_JIT_WAVES=3
    libs = [a for a in sys.argv[1:] if a.split("@")[0].endswith(".so")]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 3
    rop = "--rop" in sys.argv
    c5 = "--c5" in sys.argv  # configs[4]: the workgroup-per-reactor kernel on the 161-species stand-in
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else (4_000_000 if rop else (2048 if c5 else 16384))
    out = {lib: [] for lib in libs}
    for _ in range(reps):
        for lib in libs:
            path, *sets = lib.split("@")
            env = dict(os.environ, CKMI_LIB=os.path.abspath(path),
                       AB_TAU_REF=os.path.join(ROOT, "gpurun_out", "ab_tau_%s%s.npy" % ("c5_" if c5 else "", os.path.basename(libs[0].split("@")[0]))))
            env.update(kv.split("=", 1) for kv in sets)
            r = subprocess.run([sys.executable, "-c", (ROP_CHILD % (ROOT, n) if rop else CHILD % (ROOT, n, c5))], env=env, capture_output=True, text=True,
                               timeout=300)
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            out[lib].append(d)
            print(os.path.basename(lib), d, flush=True)
    summary = {os.path.basename(k): {"median_ms": sorted(x["ms"] for x in v)[len(v) // 2],
                                     ("states_per_s" if rop else "reactors_per_s"): n / (sorted(x["ms"] for x in v)[len(v) // 2] / 1e3)}
               for k, v in out.items()}
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
