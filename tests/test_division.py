"""The kernel divides by R = 30000 and by the QP constant n'P^-1 n = 90.00000000000153 as q = x*inv; r = fma(-q, d, x);
fma(r, inv, q) (merging_hip.hip div_const). Check on the host that this is the correctly
rounded quotient x / d, as the reference's Python division is."""

import ctypes

import numpy as np
import pytest

libm = ctypes.CDLL("libm.so.6")
libm.fma.restype = ctypes.c_double
libm.fma.argtypes = [ctypes.c_double] * 3


@pytest.mark.parametrize("d,lo,hi", [(3.0, -45.0, 45.0), (30000.0, -5e3, 2e5),
                                     (90.00000000000153, -45.0, 45.0)])
def test_fma_corrected_division_is_correctly_rounded(d, lo, hi):
    rng = np.random.default_rng(int(d))
    xs = np.concatenate([rng.uniform(lo, hi, 60000),
                         rng.uniform(-1, 1, 20000) * 2.0 ** rng.integers(-30, 30, 20000)])
    inv = 1.0 / d
    bad = 0
    for x in xs.tolist():
        q = x * inv
        r = libm.fma(-q, d, x)
        bad += libm.fma(r, inv, q) != x / d
    assert bad == 0
