"""Time ckmi_lu_factor_batched on config-5-shaped Newton matrices (n = 161) with HIP events.

    python scripts/lu_bench.py [nsys] [n]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pychemkin_amd import _native  # noqa: E402


def main():
    nsys = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 161
    g = torch.Generator(device="cuda:0").manual_seed(0)
    A0 = torch.randn((nsys, n, n), dtype=torch.float64, device="cuda:0", generator=g)
    A = torch.empty_like(A0)
    times = []
    for it in range(4):
        A.copy_(A0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _native.lu_factor_batched(A)
        e1.record()
        torch.cuda.synchronize()
        if it:
            times.append(e0.elapsed_time(e1))
    ms = sorted(times)[len(times) // 2]
    flops = nsys * 2.0 / 3.0 * n ** 3
    bytes_ = nsys * 2.0 * n * n * 8
    print(json.dumps({"nsys": nsys, "n": n, "ms": ms, "tflops": flops / ms / 1e9, "GBs": bytes_ / ms / 1e6,
                      "systems_per_s": nsys / ms * 1e3}))


if __name__ == "__main__":
    main()
