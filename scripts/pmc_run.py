"""Short fixed workload for rocprofv3 PMC passes (one reactor launch + one ROP launch).

    rocprofv3 --pmc <counters> --output-format csv -d gpurun_out/pmc_X -- python3 scripts/pmc_run.py

Reactor launch: a strided 16,384-reactor subsample of the bench sweep (configs[2]); ROP launch:
2M random (T, P, Y) states (configs[1] distribution).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402


def main():
    nr = int(os.environ.get("PMC_REACTORS", "16384"))
    ns = int(os.environ.get("PMC_STATES", "2000000"))
    mech = bench.mechanism()
    dm = _native.DeviceMechanism(mech.to_tables(), device=0)
    T0, P0, Y0, _ = bench.sweep(mech, 1, 0)
    idx = np.arange(0, len(T0), max(1, len(T0) // nr))[:nr]
    res = dm.reactor_run(_native.make_cfg(**bench.RUN), np.ones(len(idx), np.int32), T0[idx], P0[idx],
                         np.ones(len(idx)), Y0[idx])
    torch.cuda.synchronize()
    st = res["stats"].cpu().numpy()
    rng = np.random.default_rng(0)
    T = rng.uniform(300.0, 3000.0, ns)
    P = bench.P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, ns)
    Y = rng.dirichlet(0.5 * np.ones(mech.KK), ns).T.copy()
    dm.rop_thermo(T, P, Y)
    torch.cuda.synchronize()
    # configs[4] stand-in: a strided sample on the workgroup-per-reactor (MFMA) kernel
    nb = int(os.environ.get("PMC_BIG_REACTORS", "2048"))
    if nb > 0:
        bm = bench.big_mechanism()
        bdm = _native.DeviceMechanism(bm.to_tables(), device=0)
        T5, P5, Y5, pr5 = bench.sweep_c5(bm, 1, 0)
        j = np.arange(0, len(T5), max(1, len(T5) // nb))[:nb]
        r5 = bdm.reactor_run(_native.make_cfg(**bench.RUN), pr5[j], T5[j], P5[j], np.ones(len(j)), Y5[j])
        torch.cuda.synchronize()
        print(f"big reactors {len(j)} failed {int((r5['stats'][:, 6] != 0).sum().item())}")
    print(f"reactors {len(idx)} mean steps {st[:, 0].mean():.1f} failed {(st[:, 6] != 0).sum()}; rop states {ns}")


if __name__ == "__main__":
    main()
