"""Pin the CPU oracle against the reference's own outputs (golden fixtures)."""
import numpy as np
import pytest

from oracle import spgg_oracle as O
from tests._golden import Case, assert_datasets_equal, case_names


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference_bit_exact(name):
    c = Case(name)
    p = c.oracle_params()
    rs = np.random.RandomState(c.seed)
    ds, fin = O.run(p, rs, S_init=c.S_in_one)
    assert_datasets_equal(ds, c.datasets, exact=True)
    assert np.array_equal(fin["Q"], c.q_table)
    assert np.array_equal(fin["R"], c.R)
    assert np.array_equal(fin["S"], c.Sn)
    assert np.array_equal(np.array(fin["ret"], dtype=float), c.ret)
    assert fin["epsilon"] == c.epsilon
    if c.tables is not None:  # Double-Q's own tables (algorithm.q_table_1/2)
        assert np.array_equal(fin["tables"][0], c.tables[0])
        assert np.array_equal(fin["tables"][1], c.tables[1])
