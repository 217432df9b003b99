"""Element drift and failures of the configs[2] sweep and the configs[4] sample on the GPU with the element
projection on and off, and the oracle on the worst / failing reactors.   python scripts/drift_diag_r06.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from test_gpu_configs import _drift  # noqa: E402


def run(dm, T0, P0, Y0, prob, proj):
    r = dm.reactor_run(_native.make_cfg(elem_proj=proj, **bench.RUN), prob, T0, P0, np.ones(T0.size), Y0)
    return {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}


def one(name, mech, T0, P0, Y0, prob):
    dm = _native.DeviceMechanism(mech.to_tables())
    orc = Oracle(mech)
    for proj in (True, False):
        res = run(dm, T0, P0, Y0, prob, proj)
        d = _drift(mech, Y0, res["Y"])
        st = res["stats"]
        bad = np.nonzero(st[:, 6] != 0)[0]
        top = np.argsort(-d)[:5]
        print(f"== {name} proj={proj}: {T0.size} reactors, failed {bad.size} "
              f"(status {sorted(set(st[bad, 6].tolist()))}), drift p50 {np.percentile(d, 50):.2e} "
              f"p99 {np.percentile(d, 99):.2e} p99.9 {np.percentile(d, 99.9):.2e} max {d.max():.2e}", flush=True)
        for i in list(bad[:4]) + list(top):
            i = int(i)
            r, Yo = orc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), elem_proj=proj, **bench.RUN)
            do = _drift(mech, Y0[i:i + 1], Yo[None, :])[0]
            print(f"  reactor {i}: GPU status {st[i, 6]} nst {st[i, 0]} drift {d[i]:.2e} tau {res['tau'][i]:.6e} | "
                  f"oracle status {r.status} nst {r.nst} drift {do:.2e} tau {r.tau:.6e}", flush=True)


def main():
    m = bench.mechanism()
    T0, P0, Y0, prob = bench.sweep(m, 1, 0)
    one("configs[2]", m, T0, P0, Y0, prob)
    bm = bench.big_mechanism()
    T0, P0, Y0, prob = bench.sweep_c5(bm, 8, 3)
    one("configs[4] 1/8 sample", bm, T0, P0, Y0, prob)


if __name__ == "__main__":
    main()
