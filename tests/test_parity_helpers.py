"""The sliver classification of tests/parity.py on synthetic tables (CPU): an element whose relative
difference is large only because the element is tiny next to its neighbours' full crossings passes at
1e-9 (profiles/r06_parity_trace.txt), a real difference of that element does not."""
import numpy as np
import pytest

from parity import assert_parity, cartesian_neighbour_scale


def _tables(n=16, nl=3):
    rng = np.random.default_rng(0)
    b = rng.uniform(1, 2, (n ** 3, nl)) * 1e20
    a = b * (1 + rng.normal(0, 1e-12, b.shape))
    return a, b, 5 + n * 7 + n * n * 9


def test_a_sliver_passes_against_its_neighbours():
    a, b, m = _tables()
    b[m, 1] = 3.7e13
    a[m, 1] = 3.7e13 * (1 + 1.3e-7)  # the 128^3 model's cell 317912: 1.34e-7 on a sliver
    with pytest.raises(AssertionError):
        assert_parity(a, b, 1e-9, 0, "plain")
    assert_parity(a, b, 1e-9, 0, "slivers", slivers=cartesian_neighbour_scale(b, (16, 16, 16)))


def test_a_real_difference_is_not_a_sliver():
    a, b, m = _tables()
    a[m, 1] = b[m, 1] * (1 + 1e-6)  # a full crossing off by 1e-6: as large as its neighbours
    with pytest.raises(AssertionError):
        assert_parity(a, b, 1e-9, 0, "real", slivers=cartesian_neighbour_scale(b, (16, 16, 16)))


def test_neighbour_scale_stays_inside_the_grid():
    b = np.arange(8 * 2, dtype=float).reshape(8, 2)  # 2 x 2 x 2 cells, 2 wavelengths
    sc = cartesian_neighbour_scale(b, (2, 2, 2))
    # cell 0 = (0, 0, 0): face neighbours 1 (k), 2 (j), 4 (i)
    assert sc(np.array([0]), np.array([1]))[0] == max(b[1, 1], b[2, 1], b[4, 1])
