"""Newton-setup heuristics of the BDF integrator (DGMAX / MSBP / MSBJ of oracle/ckoracle.c) on a configs[2] sample,
priced with the wave kernel's phase-profile cycle costs (profiles/r06c_phase_c3.json: RHS 36.1k + Newton
iteration and its control 8.1k per call, factorisation 142.8k, Jacobian 95.9k, the rest of a step 33k cycles; the
model reproduces the profile's 121.9M cycles per reactor to 1 %).  CPU only.

    python scripts/solver_knobs_oracle.py [c5:]N name[:gcc -D flags] ...
e.g. python scripts/solver_knobs_oracle.py 512 base: dg5:-DDGMAX=0.5 bp40:-DMSBP=40
Each variant is ckoracle.c compiled with its constants made overridable (a copy in /tmp)."""
import ctypes as ct
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import oracle.oracle as oo  # noqa: E402

TMP = "/tmp/ckoracle_knobs"
os.makedirs(TMP, exist_ok=True)
src = open(os.path.join(ROOT, "oracle", "ckoracle.c")).read()
for k in ("DGMAX", "MSBP", "MSBJ", "MAXCOR", "CRDOWN", "RDIV"):
    src = re.sub(rf"^#define {k} (\S+)$", rf"#ifndef {k}\n#define {k} \1\n#endif", src, flags=re.M)
open(os.path.join(TMP, "ck.c"), "w").write(src)
open(os.path.join(TMP, "ckoracle.h"), "w").write(open(os.path.join(ROOT, "oracle", "ckoracle.h")).read())

C5 = sys.argv[1].startswith("c5:")  # "c5:N": a configs[4] sample, priced with the workgroup kernel's costs
n = int(sys.argv[1].split(":")[-1])
mech = bench.big_mechanism() if C5 else bench.mechanism()
T0, P0, Y0, prob = bench.sweep_c5(mech, 8, 3) if C5 else bench.sweep(mech, 1, 0)
idx = np.linspace(0, T0.size - 1, n).astype(np.int64)
ref = None
for v in sys.argv[2:]:
    name, _, flags = v.partition(":")
    so = os.path.join(TMP, name + ".so")
    subprocess.run(["gcc", "-O2", "-fPIC", "-fopenmp", "-shared", *flags.split(), "-o", so, os.path.join(TMP, "ck.c"), "-lm"],
                   check=True)
    oo._lib = ct.CDLL(so)
    t = time.time()
    nf, res, _ = oo.Oracle(mech).reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(n), nthreads=8,
                                               **bench.RUN)
    g = lambda k: np.array([getattr(r, k) for r in res], float)  # noqa: E731
    tau = g("tau")
    ref = tau if ref is None else ref
    nst, nfe, nje, nlu = g("nst").mean(), g("nfe").mean(), g("nje").mean(), g("nlu").mean()
    if C5:  # profiles/r06c_phase_c5.json: RHS 15.5k + solve 2.7k, RHS with J 172k, build + factor 359k, control 24.5k
        cyc = nfe * (15.5e3 + 2.7e3) + nje * 172e3 + nlu * 359e3 + nst * 24.5e3
    else:
        cyc = nfe * (36.1e3 + 8.1e3) + nlu * 142.8e3 + nje * 95.9e3 + nst * 33e3
    print(f"{name:8s} {flags:24s} fails {nf} nst {nst:.1f} nfe {nfe:.1f} nje {nje:.2f} nlu {nlu:.1f} "
          f"nef {g('nef').mean():.2f} model Mcycles {cyc / 1e6:.2f} tau max rel {np.max(np.abs(tau / ref - 1)):.1e} "
          f"{time.time() - t:.0f}s", flush=True)
