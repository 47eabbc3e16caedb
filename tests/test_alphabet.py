"""Observed alphabet and ambiguity expansion vs the reference (read_data.py:6-67)."""
import numpy as np
import pytest

from conftest import golden
from itrails_amd.read_data import column_to_index, get_idx_state, get_obs_state_dct, order_table


def test_names_match_reference():
    g = golden("alphabet.npz")
    assert list(g["names"]) == get_obs_state_dct()


def test_order_table_matches_reference():
    g = golden("alphabet.npz")
    flat, off = order_table()
    np.testing.assert_array_equal(flat, g["order_flat"])
    np.testing.assert_array_equal(off, g["order_off"])


def test_expansion_sizes():
    names = get_obs_state_dct()
    for i in (0, 255, 256, 400, 624):
        assert len(get_idx_state(i)) == 4 ** names[i].count("N")
    assert names[624] == "NNNN"


def test_column_to_index():
    assert column_to_index("aaaa") == 0
    assert column_to_index("NNNN") == 624
    with pytest.raises(ValueError):
        column_to_index("RYAA")  # IUPAC codes are not in the alphabet (read_data.py:113)
