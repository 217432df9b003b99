"""CPU A/B of the corrector's element projection (oracle/ckoracle.c elem_project): drift distribution,
and what the projection moves (tau, final T, species), on strided subsamples of configs[2] and configs[4].

    python scripts/proj_experiment.py [n_c3] [n_c5] [threads]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402


def drift(mech, Y0, Y):
    ncf = mech.ncf.astype(float)
    e0 = (Y0 / mech.wt) @ ncf.T
    e1 = (Y / mech.wt) @ ncf.T
    return np.max(np.abs(e1 - e0) / np.max(e0, axis=1, keepdims=True), axis=1)


def run(name, mech, T0, P0, Y0, prob, n, threads):
    idx = np.linspace(0, T0.size - 1, n).astype(np.int64)
    orc = Oracle(mech)
    out = {}
    for proj in (False, True):
        t = time.time()
        nf, res, Ye = orc.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(n), nthreads=threads,
                                       elem_proj=proj, **bench.RUN)
        out[proj] = (nf, np.array([r.tau for r in res]), np.array([r.T for r in res]), Ye,
                     np.array([r.nst for r in res]), time.time() - t)
    (nf0, tau0, T_0, Y_0, ns0, t0), (nf1, tau1, T_1, Y_1, ns1, t1) = out[False], out[True]
    d0, d1 = drift(mech, Y0[idx], Y_0), drift(mech, Y0[idx], Y_1)
    q = lambda d: " ".join(f"{np.percentile(d, p):.2e}" for p in (50, 90, 99, 100))
    print(f"== {name}: {n} reactors, fails {nf0} / {nf1}, wall {t0:.1f} / {t1:.1f} s")
    print(f"  drift p50 p90 p99 max   no proj: {q(d0)}")
    print(f"                          proj   : {q(d1)}")
    print(f"  max |dtau/tau| {np.max(np.abs(tau1 / tau0 - 1)):.2e}  max |dT/T| {np.max(np.abs(T_1 / T_0 - 1)):.2e}")
    big = Y_0 > 1e-6
    print(f"  species > 1e-6: max rel change {np.max(np.abs(Y_1[big] / Y_0[big] - 1)):.2e};"
          f"  > 1e-10: {np.max(np.abs(Y_1[Y_0 > 1e-10] / Y_0[Y_0 > 1e-10] - 1)):.2e}")
    print(f"  mean steps {ns0.mean():.1f} -> {ns1.mean():.1f}")


def main():
    n3 = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    n5 = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    th = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    m = bench.mechanism()
    T0, P0, Y0, prob = bench.sweep(m, 1, 0)
    run("configs[2]", m, T0, P0, Y0, prob, n3, th)
    if n5 > 0:
        bm = bench.big_mechanism()
        T0, P0, Y0, prob = bench.sweep_c5(bm, 8, 3)
        run("configs[4] sample", bm, T0, P0, Y0, prob, n5, th)


if __name__ == "__main__":
    main()
