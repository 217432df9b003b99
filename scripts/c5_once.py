"""One launch of the workgroup-per-reactor kernel on a strided sample of the configs[4] stand-in sweep
(bench.sweep_c5), for PMC passes and A/B timing.   python scripts/c5_once.py [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    m = bench.big_mechanism()
    dm = _native.DeviceMechanism(m.to_tables(), device=0)
    T0, P0, Y0, prob = bench.sweep_c5(m, 1, 0)
    idx = np.arange(0, len(T0), max(1, len(T0) // n))[:n]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    res = dm.reactor_run(_native.make_cfg(**bench.RUN), prob[idx], T0[idx], P0[idx], np.ones(len(idx)), Y0[idx])
    e1.record()
    torch.cuda.synchronize()
    st = res["stats"].cpu().numpy()
    print(f"c5 sample: {len(idx)} reactors, {e0.elapsed_time(e1):.1f} ms, mean steps {st[:, 0].mean():.1f}, "
          f"failed {(st[:, 6] != 0).sum()}")


if __name__ == "__main__":
    main()
