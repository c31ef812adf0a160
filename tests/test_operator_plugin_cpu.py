"""The RLAlgorithm plug-in point of the drop-in SPGG (reference spgg.py:111-118,
algorithms.py:44-93): built-in operators and the reference's own instances are
accepted, custom arithmetic is refused at construction with a ValueError that
names the class -- never silently replaced by the built-in operator's math."""
import sys
import types
from abc import ABC, abstractmethod

import numpy as np
import pytest

from spgg_amd import SPGG
from spgg_amd import algorithms as A


def _reference_style_module():
    """A module shaped like the reference's src/model/algorithms.py (class names, ABC
    methods, hyper-parameters), standing in for an instance built from that package."""
    mod = types.ModuleType("src.model.algorithms")

    class RLAlgorithm(ABC):
        def __init__(self, alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs):
            self.alpha, self.gamma, self.epsilon = alpha, gamma, epsilon
            self.epsilon_decay, self.epsilon_min = epsilon_decay, epsilon_min

        def decay_epsilon(self):
            self.epsilon = max(self.epsilon * self.epsilon_decay, self.epsilon_min)

        @abstractmethod
        def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
            pass

        @abstractmethod
        def select_action(self, q_table, states, L, **kwargs):
            pass

    class QLearning(RLAlgorithm):
        def select_action(self, q_table, states, L, **kwargs):
            raise AssertionError("the stand-in's arithmetic must not run")

        def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
            raise AssertionError("the stand-in's arithmetic must not run")

    class DoubleQLearning(QLearning):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.q_table_1 = self.q_table_2 = None

        def initialize_q_tables(self, shape):
            self.q_table_1 = np.random.uniform(low=-0.01, high=0.01, size=shape)
            self.q_table_2 = np.random.uniform(low=-0.01, high=0.01, size=shape)

        def get_combined_q_table(self):
            return (self.q_table_1 + self.q_table_2) / 2

    for cls in (RLAlgorithm, QLearning, DoubleQLearning):
        cls.__module__ = mod.__name__
        setattr(mod, cls.__name__, cls)
    return mod


HP = dict(alpha=0.3, gamma=0.8, epsilon=0.4, epsilon_decay=0.98, epsilon_min=0.02)


def test_builtin_instances_and_names():
    for name, cls in (("qlearning", A.QLearning), ("sarsa", A.SARSA), ("expected_sarsa", A.ExpectedSARSA),
                      ("double_qlearning", A.DoubleQLearning)):
        assert A.canonical_name(cls(**HP)) == name
        assert A.canonical_name(name) == name
    m = SPGG(L=6, iterations=3, algorithm=A.SARSA(**HP))
    assert isinstance(m.algorithm, A.SARSA)


def test_subclass_overriding_update_is_refused():
    class MyQ(A.QLearning):
        def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
            return q_table * 0

    with pytest.raises(ValueError, match=r"MyQ.*update_q_table"):
        SPGG(L=6, iterations=3, algorithm=MyQ(**HP))
    with pytest.raises(ValueError, match="MyQ"):
        A.canonical_name(MyQ(**HP))


def test_subclass_overriding_decay_is_refused():
    class Slow(A.ExpectedSARSA):
        def decay_epsilon(self):
            self.epsilon *= 0.5

    with pytest.raises(ValueError, match=r"Slow.*decay_epsilon"):
        SPGG(L=6, iterations=3, algorithm=Slow(**HP))


def test_direct_rlalgorithm_subclass_is_refused():
    class Custom(A.RLAlgorithm):
        def select_action(self, q_table, states, L, **kwargs):
            return np.zeros((L, L), dtype=int)

    class Bare(A.RLAlgorithm):
        pass

    for cls in (Custom, Bare):
        with pytest.raises(ValueError, match=cls.__name__):
            SPGG(L=6, iterations=3, algorithm=cls(**HP))


def test_state_only_subclass_is_accepted():
    class Tagged(A.DoubleQLearning):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self.tag = "run-7"

    m = SPGG(L=6, iterations=3, algorithm=Tagged(**HP))
    assert A.canonical_name(m.algorithm) == "double_qlearning"
    assert m.algorithm.q_table_1.shape == (6, 6, 2, 2)  # spgg.py:124-127 ran through the instance


def test_reference_style_instances():
    ref = _reference_style_module()
    sys.modules[ref.__name__] = ref
    try:
        q = ref.QLearning(**HP)
        np.random.seed(5)
        m = SPGG(L=6, iterations=3, algorithm=q)
        assert m.algorithm is q and A.canonical_name(q) == "qlearning"
        dq = ref.DoubleQLearning(**HP)
        m = SPGG(L=6, iterations=3, algorithm=dq)
        assert A.canonical_name(dq) == "double_qlearning"
        np.testing.assert_array_equal(m.q_table, (dq.q_table_1 + dq.q_table_2) / 2)

        class RefOverride(ref.QLearning):
            def select_action(self, q_table, states, L, **kwargs):
                return np.ones((L, L), dtype=int)

        with pytest.raises(ValueError, match=r"RefOverride.*select_action"):
            SPGG(L=6, iterations=3, algorithm=RefOverride(**HP))

        class RefCustom(ref.RLAlgorithm):
            def select_action(self, q_table, states, L, **kwargs):
                return np.ones((L, L), dtype=int)

            def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
                return q_table

        with pytest.raises(ValueError, match="RefCustom"):
            SPGG(L=6, iterations=3, algorithm=RefCustom(**HP))
    finally:
        sys.modules.pop(ref.__name__, None)


def test_same_named_class_from_another_module_is_refused():
    """A user's modified copy of the reference's algorithms.py (my/algorithms.py) defines a
    class named QLearning whose update differs: only the reference's own module path
    (src.model.algorithms) and this package's are matched, so the copy is refused instead of
    silently running the built-in operator's arithmetic."""
    mod = types.ModuleType("my.algorithms")

    class RLAlgorithm(ABC):
        def __init__(self, alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs):
            self.alpha, self.gamma, self.epsilon = alpha, gamma, epsilon
            self.epsilon_decay, self.epsilon_min = epsilon_decay, epsilon_min

    class QLearning(RLAlgorithm):
        def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
            return q_table * 0.5   # the modification

    for cls in (RLAlgorithm, QLearning):
        cls.__module__ = mod.__name__
    with pytest.raises(ValueError, match=r"my\.algorithms\..*QLearning.*update_q_table"):
        SPGG(L=6, iterations=3, algorithm=QLearning(**HP))


def test_non_operator_is_refused_like_the_reference():
    with pytest.raises(ValueError, match="algorithm must be str or RLAlgorithm"):
        SPGG(L=6, iterations=3, algorithm=3.5)
    with pytest.raises(ValueError, match="Unknown algorithm"):
        SPGG(L=6, iterations=3, algorithm="td-lambda")
