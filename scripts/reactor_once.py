"""One reactor-kernel launch over a strided subsample of the bench sweep (for profilers).

    python scripts/reactor_once.py [n]
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    mech = bench.mechanism()
    dm = _native.DeviceMechanism(mech.to_tables(), device=0)
    T0, P0, Y0, _ = bench.sweep(mech, 1, 0)
    idx = np.arange(0, len(T0), max(1, len(T0) // n))[:n]
    res = dm.reactor_run(_native.make_cfg(**bench.RUN), np.ones(len(idx), np.int32), T0[idx], P0[idx],
                         np.ones(len(idx)), Y0[idx])
    torch.cuda.synchronize()
    print("steps", float(res["stats"][:, 0].float().mean().item()))


if __name__ == "__main__":
    main()
