"""The oracle deep into a runner-shaped run: SPGG(L=100, iterations=10001) of the reference
(tests/golden/make_deep_golden.py, the reference itself in the survey container), through
the snapshot iterations 5000 and 10000 (spgg.py:153,397-402) -- every dataset, the final
Q / R / S and the return value.  Bit-exact: the oracle and the reference run the same
NumPy operations in the same order."""
import numpy as np

from oracle import spgg_oracle as O
from tests._golden import DeepDigest, _PARAM_KEYS


def test_oracle_matches_reference_deep_run():
    d = DeepDigest()
    p = O.Params(**{k: v for k, v in d.kwargs.items() if k in _PARAM_KEYS})
    rs = np.random.RandomState(d.seed)
    ds, fin = O.run(p, rs)
    assert d.meta["iterations_recorded"] == 10001 and "R_snapshot_10000" in ds and "Sn_snapshot_5000" in ds
    key = rs.get_state()
    d.check(ds, fin["Q"], fin["R"], fin["S"], fin["ret"], rtol=0, atol=0, mt_key=key[1])
    assert int(key[2]) == d.meta["mt_pos"]
    assert fin["epsilon"] == d.meta["epsilon"]
