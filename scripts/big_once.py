"""Quick check of the workgroup-per-reactor kernel on the 161-species stand-in (a few reactors,
bounded steps) against the oracle.  python scripts/big_once.py [n] [t_end]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from conftest import BIG_CHEM, BIG_THERM  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from pychemkin_amd.mechanism import Mechanism  # noqa: E402
from test_gpu_bigreactor import _cases, tracer_Y  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    t_end = float(sys.argv[2]) if len(sys.argv) > 2 else 2e-3
    m = Mechanism.from_files(BIG_CHEM, BIG_THERM)
    dm = _native.DeviceMechanism(m.to_tables())
    T0, P0, phi, prob = _cases(n, 11)
    Y0 = tracer_Y(m, phi)
    run = dict(energy=1, t_end=t_end, atol=1e-10, rtol=1e-8, ign_mode="TIFP", max_steps=5000)
    t = time.time()
    res = dm.reactor_run(_native.make_cfg(**run), prob, T0, P0, np.ones(n), Y0)
    torch.cuda.synchronize()
    dt = time.time() - t
    res = {k: v.cpu().numpy() for k, v in res.items() if not k.startswith("_")}
    orc = Oracle(m)
    _, ref, _ = orc.reactor_batch(T0, P0, Y0, problem=prob, V0=np.ones(n), **run)
    print(f"{n} reactors in {dt:.3f} s")
    for i in range(n):
        r = ref[i]
        print(i, "gpu tau %.6e T %.6f stats %s | oracle tau %.6e T %.6f nst %d nlu %d status %d" % (
            res["tau"][i], res["T"][i], res["stats"][i].tolist(), r.tau, r.T, r.nst, r.nlu, r.status))


if __name__ == "__main__":
    main()
