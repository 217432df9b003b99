"""Element drift of the configs[4] sample (tests/test_gpu_configs.py::test_configs4_sample's run) on the GPU:
the worst reactors and a named one.   python scripts/c5_drift_top.py [reactor]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from pychemkin_amd import _native  # noqa: E402
from test_gpu_configs import _drift, _run  # noqa: E402

m = bench.big_mechanism()
dm = _native.DeviceMechanism(m.to_tables())
T0, P0, Y0, prob = bench.sweep_c5(m, 8, 3)
res = _run(dm, T0, P0, Y0, prob)
d = _drift(m, Y0, res["Y"])
top = np.argsort(-d)[:8]
print("worst:", [(int(i), float(d[i])) for i in top])
print("percentiles 50/99/99.9:", [float(np.percentile(d, q)) for q in (50, 99, 99.9)])
if len(sys.argv) > 1:
    w = int(sys.argv[1])
    print("reactor", w, float(d[w]))
