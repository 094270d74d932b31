"""CERES_TRI_CHAIN (render_hip.hip tri_test / tri_mask): Möller–Trumbore's acceptance
(u >= 0) & (v >= 0) & (w >= 0) & (t >= tmin) & (t <= tmax) (triangle.hpp:95-115) evaluated as a
chain of selects -- x1 = u >= 0 ? v : -1, x2 = x1 >= 0 ? w : -1, x3 = x2 >= 0 ? t : -1,
accept = (x3 >= tmin) & (x3 <= tmax) -- is the same predicate for every float input when
tmin > -1 (the kernels use tmin = 0).  Checked on random floats of every magnitude and on all
combinations of the special values (+-0, +-inf, NaN, +-denormal, +-1)."""
import itertools

import numpy as np


def conj(u, v, w, t, tmin, tmax):
    return (u >= 0) & (v >= 0) & (w >= 0) & (t >= tmin) & (t <= tmax)


def chain(u, v, w, t, tmin, tmax):
    m1 = np.float32(-1.0)
    x1 = np.where(u >= 0, v, m1)
    x2 = np.where(x1 >= 0, w, m1)
    x3 = np.where(x2 >= 0, t, m1)
    return (x3 >= tmin) & (x3 <= tmax)


def test_chain_equals_conjunction_on_random_floats():
    rng = np.random.default_rng(5)
    n = 4_000_000
    # random bit patterns (every magnitude, NaNs and infinities included) and small signed values
    bits = rng.integers(0, 2**32, size=(4, n), dtype=np.uint64).astype(np.uint32).view(np.float32)
    small = rng.normal(size=(4, n)).astype(np.float32)
    with np.errstate(invalid="ignore"):
        for arr in (bits, small):
            for tmin, tmax in ((np.float32(0), np.float32(np.finfo(np.float32).max)), (np.float32(0), np.float32(1.5))):
                np.testing.assert_array_equal(chain(*arr, tmin, tmax), conj(*arr, tmin, tmax))


def test_chain_equals_conjunction_on_special_values():
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.0, -1.0, 0.5, -0.5], np.float32)
    combos = np.array(list(itertools.product(sp, repeat=4)), np.float32).T
    with np.errstate(invalid="ignore"):
        for tmax in (np.float32(np.finfo(np.float32).max), np.float32(0.5), np.float32(0.0)):
            np.testing.assert_array_equal(chain(*combos, np.float32(0), tmax), conj(*combos, np.float32(0), tmax))
