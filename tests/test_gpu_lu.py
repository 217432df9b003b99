"""Batched MFMA LU (ckmi_lu_factor_batched / ckmi_lu_solve_batched) against LAPACK dgetrf/dgetrs.

The checker is scipy's LAPACK (the reference's Chemkin links MKL LAPACK for the same
factorisation, chemkin_wrapper.py:215-228): pivots must agree exactly, factors within a few
ulps of the matrix scale (different summation order: blocked MFMA tiles vs LAPACK's
recursive panels), solutions within 1e-12 relative.
"""
import numpy as np
import pytest
import scipy.linalg as sla

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


def _factor(A_np):
    import torch
    from pychemkin_amd import _native

    A = torch.as_tensor(A_np.copy(), device="cuda:0")
    _, ipiv, info = _native.lu_factor_batched(A)
    torch.cuda.synchronize()
    return A.cpu().numpy(), ipiv.cpu().numpy(), info.cpu().numpy()


def _newton_like(rng, nsys, n):
    """I - gamma J with a chemistry-like spread of magnitudes (stiff, not diagonally dominant)."""
    J = rng.standard_normal((nsys, n, n)) * 10.0 ** rng.uniform(-3, 6, (nsys, n, n))
    gamma = 10.0 ** rng.uniform(-9, -5, (nsys, 1, 1))
    return np.eye(n)[None] - gamma * J


@pytest.mark.parametrize("n", [1, 5, 16, 17, 54, 100, 161, 192])
def test_lu_matches_lapack(n):
    rng = np.random.default_rng(n)
    nsys = 24
    A = rng.standard_normal((nsys, n, n))
    A[: nsys // 2] = _newton_like(rng, nsys // 2, n)
    LU, piv, info = _factor(A)
    assert np.all(info == 0)
    for s in range(nsys):
        lu_ref, piv_ref = sla.lu_factor(A[s])
        np.testing.assert_array_equal(piv[s], piv_ref)
        scale = np.abs(lu_ref).max()
        np.testing.assert_allclose(LU[s], lu_ref, rtol=0, atol=1e-12 * scale)
        # P L U reconstructs A
        L = np.tril(LU[s], -1) + np.eye(n)
        U = np.triu(LU[s])
        PA = A[s].copy()
        for i, p in enumerate(piv[s]):
            PA[[i, p]] = PA[[p, i]]
        np.testing.assert_allclose(L @ U, PA, rtol=0, atol=1e-13 * np.abs(A[s]).max() * n)


@pytest.mark.parametrize("n", [54, 161])
def test_lu_solve(n):
    import torch
    from pychemkin_amd import _native

    rng = np.random.default_rng(7 + n)
    nsys = 64
    A = _newton_like(rng, nsys, n)
    b = rng.standard_normal((nsys, n))
    At = torch.as_tensor(A.copy(), device="cuda:0")
    _, ipiv, info = _native.lu_factor_batched(At)
    bt = torch.as_tensor(b.copy(), device="cuda:0")
    _native.lu_solve_batched(At, ipiv, bt)
    x = bt.cpu().numpy()
    assert np.all(info.cpu().numpy() == 0)
    for s in range(nsys):
        xr = np.linalg.solve(A[s], b[s])
        np.testing.assert_allclose(x[s], xr, rtol=1e-10, atol=1e-12 * np.abs(xr).max())


def test_lu_singular_and_edge_cases():
    import torch
    from pychemkin_amd import _native

    rng = np.random.default_rng(3)
    n = 40
    A = rng.standard_normal((3, n, n))
    A[1, :, 7] = 0.0  # zero column: U(7,7) = 0 exactly, dgetrf info = 8
    A[2] = 0.0
    LU, piv, info = _factor(A)
    assert info[0] == 0 and info[1] == 8 and info[2] == 1
    assert piv[1][7] == 7  # all-zero pivot column: no interchange (idamax picks the first entry)
    # empty batch and size limits
    E = torch.empty((0, 8, 8), dtype=torch.float64, device="cuda:0")
    _native.lu_factor_batched(E)
    with pytest.raises(ValueError):
        _native.lu_factor_batched(torch.zeros((1, 193, 193), dtype=torch.float64, device="cuda:0"))


def test_lu_batch_order_invariance():
    """Each matrix's factors do not depend on its batch neighbours or position (bitwise)."""
    rng = np.random.default_rng(11)
    A = _newton_like(rng, 40, 161)
    LU1, p1, _ = _factor(A)
    perm = rng.permutation(40)
    LU2, p2, _ = _factor(A[perm])
    np.testing.assert_array_equal(LU2, LU1[perm])
    np.testing.assert_array_equal(p2, p1[perm])
