"""Per-reactor solver statistics of the c3 sweep (configs[2]) for a queue / tail-effect analysis:
writes gpurun_out/c3_stats.npz (stats[n][8], kernel ms) -- diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402

mech = bench.mechanism()
dm = _native.DeviceMechanism(mech.to_tables(), device=0)
T0, P0, Y0, prob = bench.sweep(mech, 1, 0)
cfg = _native.make_cfg(**bench.RUN)
args = (prob, T0, P0, np.ones(len(T0)), Y0)
dm.reactor_run(cfg, *args)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
res = dm.reactor_run(cfg, *args)
e1.record()
torch.cuda.synchronize()
np.savez(os.path.join(ROOT, "gpurun_out", "c3_stats.npz"), stats=res["stats"].cpu().numpy(), T0=T0, P0=P0,
         ms=e0.elapsed_time(e1))
print("ms", e0.elapsed_time(e1))
