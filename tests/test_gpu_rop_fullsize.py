"""configs[1] at its full size: 10M GRI-3.0 states through the specialised ROP kernel in one launch.

The oracle cannot evaluate 10M states in test time, so the full launch is checked through properties
that hold for every state whatever the rates are, plus an oracle comparison on a stride sample that
spans the whole launch (first and last state included):
  * element conservation: sum_k n_ek wdot_k = 0 for every element e (relative to sum_k n_ek |wdot_k|);
  * mass conservation: sum_k W_k wdot_k = 0 (relative to sum_k W_k |wdot_k|);
  * every output finite, cp > 0;
  * determinism: a second launch gives bitwise the same wdot / cp / h (checksum of checksums);
  * 4,096 strided states within 1e-11 of the oracle (the small-batch bar of test_gpu_rop_jit.py).
Tolerance of the conservation checks: 1e-12 -- each wdot_k is a signed sum of rates of progress
whose cancellation error is a few ulps of the largest term.
"""
import numpy as np
import pytest

from conftest import P_ATM

pytestmark = pytest.mark.gpu

NS = 10_000_000


def test_rop_10m_states_conserve_and_match_oracle_sample(tables, oracle, mech):
    import torch

    from pychemkin_amd import _native

    _native.set_rop_path(2)  # the specialised kernel (the bench's configs[1] kernel)
    try:
        dev = "cuda:0"
        dm = _native.DeviceMechanism(tables)
        g = torch.Generator(device=dev).manual_seed(1234)
        T = 300.0 + 2700.0 * torch.rand(NS, dtype=torch.float64, device=dev, generator=g)
        P = P_ATM * 10.0 ** (-1.0 + 3.0 * torch.rand(NS, dtype=torch.float64, device=dev, generator=g))
        Y = torch.rand((mech.KK, NS), dtype=torch.float64, device=dev, generator=g) ** 4  # skewed, some tiny
        Y /= Y.sum(dim=0, keepdim=True)
        w, cp, h = dm.rop_thermo(T, P, Y)
        torch.cuda.synchronize()

        assert bool(torch.isfinite(w).all()) and bool(torch.isfinite(cp).all()) and bool(torch.isfinite(h).all())
        assert bool((cp > 0).all())

        ncf = torch.as_tensor(mech.ncf.astype(np.float64), device=dev)  # [MM][KK]
        wt = torch.as_tensor(mech.wt, device=dev)
        for lo in range(0, NS, 1_000_000):  # in slices: [MM][1M] temporaries
            ws = w[:, lo:lo + 1_000_000]
            el = (ncf @ ws).abs() / (ncf @ ws.abs()).clamp_min(1e-300)
            assert float(el.max()) < 1e-12
            ms = (wt @ ws).abs() / (wt @ ws.abs()).clamp_min(1e-300)
            assert float(ms.max()) < 1e-12

        w2, cp2, h2 = dm.rop_thermo(T, P, Y)
        assert torch.equal(w, w2) and torch.equal(cp, cp2) and torch.equal(h, h2)

        idx = np.unique(np.r_[np.linspace(0, NS - 1, 4096).astype(np.int64), NS - 1])
        ti = torch.as_tensor(idx, device=dev)
        Ts, Ps, Ys = T[ti].cpu().numpy(), P[ti].cpu().numpy(), Y[:, ti].cpu().numpy()
        wo, cpo, ho = oracle.rop_batch(Ts, Ps, Ys)
        wg = w[:, ti].cpu().numpy()
        scale = np.max(np.abs(wo), axis=0, keepdims=True)
        assert np.max(np.abs(wg - wo) / scale) < 1e-11
        assert np.max(np.abs(cp[ti].cpu().numpy() / cpo - 1)) < 1e-12
    finally:
        _native.set_rop_path(0)
