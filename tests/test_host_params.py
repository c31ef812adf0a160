"""Host-side parameter logic (CPU only): constants the device consumes."""
import numpy as np
import pytest

from spgg_amd.engine import ReplicaParams, epsilon_table
from oracle import spgg_oracle as O


@pytest.mark.parametrize("gain,loss,rmin,rmax,unit", [
    (1.0, 1, -10, 10, 1.0), (0.5, 1, -10, 10, 0.5), (0.25, 0.5, -1, 1, 0.25),
    (0.3, 1, -10, 10, None), (1.0, 1, -200, 10, None), (1, 1, 5, 10, None), (1.0, 1.0, 10, -10, None)])
def test_rep_unit(gain, loss, rmin, rmax, unit):
    p = ReplicaParams(rep_gain_C=gain, delta_R_D=loss, R_min=rmin, R_max=rmax)
    assert p.rep_unit() == unit
    if unit is not None:
        c = p.to_c()
        assert c.rk_gain * unit == gain and c.rk_loss * unit == loss
        assert c.rk_min * unit == rmin and c.rk_max * unit == rmax


@pytest.mark.parametrize("r,c,cost", [(3.0, 1, 1), (2, 1, 0.5), (3.6, 1.0, 1.0), (5.0, 2, 0.3)])
def test_payoff_tables_match_reference_arithmetic(r, c, cost):
    """pay_c/pay_d[N] equal the reference's ((r*c*N/5 - cost)*S0 + (r*c*N/5)*S1) (spgg.py:256-257)."""
    p = ReplicaParams(r=r, c=c, cost=cost).to_c()
    for N in range(6):
        Na = np.array([N])
        coop = (r * c * Na / 5 - cost) * np.array([1]) + (r * c * Na / 5) * np.array([0])
        defe = (r * c * Na / 5 - cost) * np.array([0]) + (r * c * Na / 5) * np.array([1])
        assert p.pay_c[N] == coop[0] and p.pay_d[N] == defe[0]
    assert p.norm_min == r - 5 and p.norm_den == 4 * r - (r - 5)


def test_epsilon_table_matches_oracle_schedule():
    o = O.Params(epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01)
    tab = epsilon_table(0.5, 0.99, 0.01, 600)
    assert np.array_equal(tab[1:601], O.epsilon_schedule(o, 600))
