"""The oracle's batched dense LU (bench.py's LU-line CPU baseline and the GPU LU tests' checker) against
LAPACK dgetrf via scipy: same pivots, same factors, singular systems flagged."""
import numpy as np
import scipy.linalg as sl

from oracle.oracle import lu_factor_batch


def test_lu_factor_batch_matches_lapack():
    rng = np.random.default_rng(3)
    n = 47
    A = np.eye(n) - 1e-3 * rng.standard_normal((6, n, n)) * 10.0 ** (4.0 * rng.random((6, n, n)))
    LU, piv, info = lu_factor_batch(A, 2)
    assert (info == 0).all()
    for s in range(A.shape[0]):
        lu, p = sl.lu_factor(A[s])
        assert (piv[s] == p).all()
        np.testing.assert_allclose(LU[s], lu, rtol=0, atol=1e-12 * np.abs(lu).max())


def test_lu_factor_batch_singular_and_empty():
    A = np.zeros((2, 5, 5))
    A[1] = np.eye(5)
    A[0, :, 2] = 0.0
    A[0] += np.diag([1.0, 2.0, 0.0, 4.0, 5.0])
    _, _, info = lu_factor_batch(A)
    assert info[0] == 3 and info[1] == 0
    LU, piv, info = lu_factor_batch(np.zeros((0, 4, 4)))
    assert LU.shape == (0, 4, 4) and info.shape == (0,)
