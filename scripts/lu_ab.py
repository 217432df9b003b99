"""A/B timing of ckmi_lu_factor_batched builds: python scripts/lu_ab.py lib1.so [lib2.so ...]

Each library is a standalone build of csrc/ckmi_lu.hip (scripts/lu_ab_build.sh); timing only."""
import ctypes as ct
import json
import sys

import torch


def time_lib(path, nsys=16384, n=161, reps=4, newton=False):
    lib = ct.CDLL(path)
    lib.ckmi_lu_factor_batched.argtypes = [ct.c_int32, ct.c_int32, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    g = torch.Generator(device="cuda:0").manual_seed(0)
    A0 = torch.randn((nsys, n, n), dtype=torch.float64, device="cuda:0", generator=g)
    if newton:  # I - gamma J with J entries spread over 6 decades (bench.py lu_bench)
        A0 = torch.eye(n, dtype=torch.float64, device="cuda:0") - 1e-6 * A0 * 10.0 ** (6.0 * torch.rand(
            (nsys, n, n), dtype=torch.float64, device="cuda:0", generator=g))
    A = torch.empty_like(A0)
    ipiv = torch.empty((nsys, n), dtype=torch.int32, device="cuda:0")
    info = torch.empty(nsys, dtype=torch.int32, device="cuda:0")
    ts = []
    for it in range(reps):
        A.copy_(A0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = lib.ckmi_lu_factor_batched(nsys, n, A.data_ptr(), ipiv.data_ptr(), info.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if it:
            ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2], A.cpu(), ipiv.cpu(), info.cpu()


if __name__ == "__main__":
    for newton in (False, True):
        ref = None
        for p in sys.argv[1:]:
            ms, A, ipiv, info = time_lib(p, newton=newton)
            same = piv_same = maxdiff = None
            if ref is None:
                ref = (A, ipiv, info)
            else:
                same = bool(torch.equal(A, ref[0]) and torch.equal(ipiv, ref[1]) and torch.equal(info, ref[2]))
                piv_same = bool(torch.equal(ipiv, ref[1]))
                maxdiff = float(((A - ref[0]).abs().max() / ref[0].abs().max()).item())
            print(json.dumps({"lib": p, "matrices": "newton" if newton else "randn", "ms": ms,
                              "bitwise_equal_to_first": same, "pivots_equal": piv_same,
                              "max_rel_diff": maxdiff}), flush=True)
