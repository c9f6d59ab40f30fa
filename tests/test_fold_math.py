"""CPU check of the decimation-in-frequency split the N = 4096 operator uses (fft2.hip k_rowsf /
k_colsf_ip, F = 2; F = 4 was an earlier form): a column transform of N points as F transforms of L = N / F points over folded rows,
    X[F m + b] = sum_{n < L} z_b[n] w_L^(n m),   z_b[n] = w_N^(n b) sum_{r < F} a[n + L r] w_F^(r b),
with w = exp(+2 pi i / .) (the inverse transform of IFFT.compute), and the incremental radix-4 fold
order of the F = 4 row launch (rows r = 0, 2, 1, 3: s0, d0 = a0 +- a2, then z_0 = s0 + s1, z_2 = s0 - s1,
z_1 = d0 + i d1, z_3 = d0 - i d1).  float64 numpy against N * ifft."""
import numpy as np
import pytest


def fold_transform(a, F):
    N = a.shape[0]
    L = N // F
    n = np.arange(L)
    out = np.empty(N, dtype=complex)
    rows = [a[n + L * r] for r in range(F)]
    if F == 4:  # k_rowsf's incremental order
        s0, d0 = rows[0] + rows[2], rows[0] - rows[2]
        s1, d1 = rows[1] + rows[3], 1j * (rows[1] - rows[3])
        zs = [s0 + s1, d0 + d1, s0 - s1, d0 - d1]
    else:
        zs = [rows[0] + rows[1], rows[0] - rows[1]]
    for b in range(F):
        z = zs[b] * np.exp(2j * np.pi * n * b / N)
        out[F * np.arange(L) + b] = L * np.fft.ifft(z)  # sum_n z[n] w_L^(n m)
    return out


@pytest.mark.parametrize("N,F", [(64, 2), (64, 4), (4096, 2), (4096, 4)])
def test_fold_equals_column_transform(N, F):
    rng = np.random.default_rng(N + F)
    a = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    want = N * np.fft.ifft(a)
    got = fold_transform(a, F)
    assert np.max(np.abs(got - want)) <= 1e-9 * np.max(np.abs(want))


def test_fold_generic_radix_matches_incremental():
    """The generic fold sum_r a[n + L r] w_F^(r b) equals the incremental butterflies k_rowsf forms."""
    rng = np.random.default_rng(5)
    N, F = 256, 4
    L = N // F
    a = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    n = np.arange(L)
    for b in range(F):
        generic = sum(a[n + L * r] * np.exp(2j * np.pi * r * b / F) for r in range(F))
        rows = [a[n + L * r] for r in range(F)]
        s0, d0 = rows[0] + rows[2], rows[0] - rows[2]
        s1, d1 = rows[1] + rows[3], 1j * (rows[1] - rows[3])
        inc = [s0 + s1, d0 + d1, s0 - s1, d0 - d1][b]
        np.testing.assert_allclose(inc, generic, rtol=0, atol=1e-12)
