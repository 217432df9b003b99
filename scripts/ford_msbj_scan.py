"""FORD robustness of the Jacobian refresh interval: the five FORD reactors of tests/test_ford.py over many
rtol perturbations, the oracle built with -DMSBJ=<m> from scripts/solver_knobs_oracle.py's overridable copy
(/tmp/ckoracle_knobs/ck.c; run that script once first).   python scripts/ford_msbj_scan.py 50 15 ..."""
import sys, ctypes as ct, subprocess
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import oracle.oracle as oo
from test_ford import FORD_CHEM, THERM
from conftest import P_ATM, ch4_air_Y
from pychemkin_amd.mechanism import Mechanism
fm = Mechanism.from_files(FORD_CHEM, THERM)
cases = [(1200, 1, 1.0, 1), (1400, 10, 1.0, 2), (1100, 0.5, 0.7, 1), (1600, 50, 1.5, 1), (1300, 30, 0.5, 2)]
rts = ([1e-8 * (1 + 0.01 * k) for k in range(-10, 11)] + [1e-7, 1e-9, 3e-8, 3e-9]
       + [1e-8 * (1 + 0.002 * k + 0.0007) for k in range(-25, 25)] + [3e-9 * (1 + 0.01 * k) for k in range(-5, 6)])
for msbj in sys.argv[1:]:
    so = f"/tmp/ckoracle_knobs/f{msbj}.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-fopenmp", "-shared", f"-DMSBJ={msbj}", "-o", so, "/tmp/ckoracle_knobs/ck.c", "-lm"], check=True)
    oo._lib = ct.CDLL(so)
    orc = oo.Oracle(fm)
    bad, ns = [], []
    for rt in rts:
        for T0, p, phi, prob in cases:
            r, _ = orc.reactor(float(T0), p * P_ATM, 1.0, ch4_air_Y(fm, phi)[0], problem=prob, energy=1, t_end=1.0, atol=1e-10, rtol=rt, ign_mode="TIFP")
            if r.status != 0 or r.nst >= 2500: bad.append((T0, p, phi, prob, "%.4g" % rt, r.status, r.nst))
            else: ns.append(r.nst)
    print("MSBJ", msbj, "runs", len(rts) * len(cases), "bad", len(bad), bad[:3], "mean nst %.0f max %d" % (np.mean(ns), max(ns)), flush=True)
