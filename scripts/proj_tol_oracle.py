"""Oracle drift / step counts on a configs[4] sample for a ckoracle.c build with other PROJ_TOL / PROJ_EVERY
(gcc -O2 -fPIC -fopenmp -shared -DPROJ_TOL=1e-4 -DPROJ_EVERY=4 -o /tmp/x.so oracle/ckoracle.c -lm).
    python scripts/proj_tol_oracle.py {default|/tmp/x.so} N"""
import sys, time, ctypes as ct
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import oracle.oracle as oo
variant = sys.argv[1]
if variant != "default":
    oo._lib = ct.CDLL(variant)
import bench
from test_gpu_configs import _drift
bm = bench.big_mechanism()
T0, P0, Y0, prob = bench.sweep_c5(bm, 8, 3)
n = int(sys.argv[2])
idx = np.linspace(0, T0.size - 1, n).astype(np.int64)
orc = oo.Oracle(bm)
t = time.time()
nf, res, Ye = orc.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(n), nthreads=8, **bench.RUN)
d = _drift(bm, Y0[idx], Ye)
st = np.array([r.status for r in res]); ns = np.array([r.nst for r in res])
print(variant, "fails", nf, "status", sorted(set(st.tolist())), "drift p50 %.2e p99 %.2e max %.2e" % (np.percentile(d,50), np.percentile(d,99), d.max()), "mean nst %.1f max nst %d" % (ns.mean(), ns.max()), "%.1fs" % (time.time()-t))
