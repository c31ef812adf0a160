"""RL operator interface of the reference (src/model/algorithms.py:10-383).

The classes keep the reference's constructor signature, attributes, eps
schedule (`decay_epsilon`, algorithms.py:40-42) and the `create_algorithm`
factory with its ValueError.  Their per-lattice `select_action` /
`update_q_table` arithmetic is fused into the HIP step (libspgg_hip.so) and
driven by `SPGG.run` / `BatchEngine`; calling those two methods on their own
raises, because this package has no NumPy execution path by design.

The plug-in point (`SPGG(algorithm=<RLAlgorithm instance>)`, spgg.py:111-118):
`operator_kind` accepts these four classes, the reference's own four (an
instance built from src/model/algorithms.py drops in) and subclasses that only
add state; anything that redefines the operator's methods is refused with a
ValueError naming the class, so custom arithmetic can never silently run as the
built-in operator.

GPU coverage: all four operators -- QLearning (algorithms.py:96-133), SARSA
(:136-178), ExpectedSARSA (:181-234), DoubleQLearning (:237-341) -- each a
template instance of the step kernel (spgg_kernels.hip, SPGG_ALG_*).
"""
from __future__ import annotations

from abc import ABC
from typing import Tuple

import numpy as np


class RLAlgorithm(ABC):
    """Base class (algorithms.py:10-93)."""

    kind = "abstract"

    def __init__(self, alpha: float, gamma: float, epsilon: float,
                 epsilon_decay: float, epsilon_min: float, **kwargs):
        self.alpha = alpha
        self.gamma = gamma
        self.epsilon = epsilon
        self.epsilon_decay = epsilon_decay
        self.epsilon_min = epsilon_min

    def decay_epsilon(self):
        """algorithms.py:40-42 (host scalar; the device reads the same schedule)."""
        self.epsilon = max(self.epsilon * self.epsilon_decay, self.epsilon_min)

    def select_action(self, q_table, states, L, **kwargs):
        raise NotImplementedError(
            f"{type(self).__name__}.select_action is fused into the HIP step; drive it "
            "through SPGG.run() or BatchEngine")

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        raise NotImplementedError(
            f"{type(self).__name__}.update_q_table is fused into the HIP step; drive it "
            "through SPGG.run() or BatchEngine")


class QLearning(RLAlgorithm):
    """Off-policy TD with max over next-state actions (algorithms.py:96-133)."""
    kind = "qlearning"


class SARSA(RLAlgorithm):
    """On-policy TD (algorithms.py:136-178)."""
    kind = "sarsa"


class ExpectedSARSA(RLAlgorithm):
    """Expected-value TD under the eps-greedy policy (algorithms.py:181-234)."""
    kind = "expected_sarsa"


class DoubleQLearning(RLAlgorithm):
    """Two Q tables (algorithms.py:237-341)."""
    kind = "double_qlearning"

    def __init__(self, alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs):
        super().__init__(alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs)
        self.q_table_1 = None
        self.q_table_2 = None

    def initialize_q_tables(self, shape: Tuple[int, ...]):
        """Two more U(-0.01, 0.01) tables from the global stream (algorithms.py:250-260)."""
        self.q_table_1 = np.random.uniform(low=-0.01, high=0.01, size=shape)
        self.q_table_2 = np.random.uniform(low=-0.01, high=0.01, size=shape)

    def get_combined_q_table(self):
        """Average of both tables (algorithms.py:262-266)."""
        if self.q_table_1 is None or self.q_table_2 is None:
            raise ValueError("Q-tables not initialized. Call initialize_q_tables first.")
        return (self.q_table_1 + self.q_table_2) / 2


_ALIASES = {"qlearning": "qlearning", "q-learning": "qlearning", "sarsa": "sarsa",
            "expected_sarsa": "expected_sarsa", "expected-sarsa": "expected_sarsa",
            "double_qlearning": "double_qlearning", "double-q-learning": "double_qlearning"}

# Modules whose operator classes the device step reproduces: this module, and the reference's
# src/model/algorithms.py under the package path its scripts import it by
# (scripts/run_experiments.py:10-13 puts the repository root on sys.path: src.model.algorithms).
# A class of the same name from any other module -- a user's modified copy -- is not matched.
_OPERATOR_MODULES = (__name__, "src.model.algorithms")
# The reference's operator classes (algorithms.py:96, 136, 181, 237) by class name.
_BUILTIN_CLASSES = {"QLearning": "qlearning", "SARSA": "sarsa", "ExpectedSARSA": "expected_sarsa",
                    "DoubleQLearning": "double_qlearning"}
# Methods whose arithmetic the device step reproduces: a class that redefines any of them
# computes something the HIP kernels do not (algorithms.py:40-93, 250-341).
_FUSED_METHODS = ("select_action", "update_q_table", "decay_epsilon", "initialize_q_tables",
                  "get_combined_q_table")
_HYPER = ("alpha", "gamma", "epsilon", "epsilon_decay", "epsilon_min")


def operator_kind(algorithm) -> str:
    """Operator kind of an RLAlgorithm instance -- the reference's plug-in point
    (spgg.py:111-118) -- or ValueError when the device step cannot run it.

    Accepted: this module's four operator classes, the reference's own four
    (matched by class name and the fully qualified module src.model.algorithms, so an
    instance built from the reference package drops in), and subclasses of either that add state
    but redefine none of the operator's methods.  A subclass that overrides
    select_action / update_q_table / decay_epsilon (or Double-Q's table methods), or
    an RLAlgorithm that derives from none of the four, defines arithmetic the HIP
    step does not contain: it is refused here rather than silently replaced by the
    built-in operator's math."""
    cls = type(algorithm)
    base = None
    for k in cls.__mro__:
        if k.__module__ in _OPERATOR_MODULES and k.__name__ in _BUILTIN_CLASSES:
            base = k
            break
        if k.__name__ == "RLAlgorithm" or k is object:
            break
        redefined = [m for m in _FUSED_METHODS if m in vars(k)]
        if redefined:
            raise ValueError(
                f"algorithm {cls.__module__}.{cls.__qualname__}: {k.__qualname__} redefines "
                f"{', '.join(redefined)}; the MI355X step fuses the reference operators' own "
                f"select_action/update_q_table arithmetic (QLearning, SARSA, ExpectedSARSA, "
                f"DoubleQLearning) and cannot run a custom operator")
    if base is None:
        raise ValueError(
            f"algorithm {cls.__module__}.{cls.__qualname__} is not one of the operators the MI355X "
            f"step implements (QLearning, SARSA, ExpectedSARSA, DoubleQLearning or a subclass that "
            f"keeps their methods)")
    missing = [h for h in _HYPER if not hasattr(algorithm, h)]
    if missing:
        raise ValueError(f"algorithm {cls.__qualname__} lacks {', '.join(missing)}")
    return _BUILTIN_CLASSES[base.__name__]


def is_operator(algorithm) -> bool:
    """An RLAlgorithm of this package or an instance of the reference's RLAlgorithm
    hierarchy (duck-typed by class name: the reference package is not imported)."""
    if isinstance(algorithm, RLAlgorithm):
        return True
    return any(k.__name__ == "RLAlgorithm" and k.__module__.split(".")[-1] == "algorithms"
               for k in type(algorithm).__mro__)


def canonical_name(algorithm) -> str:
    """Operator kind of a name (create_algorithm's accepted spellings, algorithms.py:371-383)
    or of an RLAlgorithm instance (operator_kind)."""
    if not isinstance(algorithm, str) and is_operator(algorithm):
        return operator_kind(algorithm)
    name = str(algorithm).lower()
    if name not in _ALIASES:
        raise ValueError(f"Unknown algorithm: {name}. "
                         f"Supported: 'qlearning', 'sarsa', 'expected_sarsa', 'double_qlearning'")
    return _ALIASES[name]


def create_algorithm(algorithm_name: str, alpha: float, gamma: float,
                     epsilon: float, epsilon_decay: float, epsilon_min: float,
                     **kwargs) -> RLAlgorithm:
    """Factory with the reference's accepted names and error (algorithms.py:344-383)."""
    algorithm_name = algorithm_name.lower()
    if algorithm_name in ("qlearning", "q-learning"):
        return QLearning(alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs)
    if algorithm_name == "sarsa":
        return SARSA(alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs)
    if algorithm_name in ("expected_sarsa", "expected-sarsa"):
        return ExpectedSARSA(alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs)
    if algorithm_name in ("double_qlearning", "double-q-learning"):
        return DoubleQLearning(alpha, gamma, epsilon, epsilon_decay, epsilon_min, **kwargs)
    raise ValueError(f"Unknown algorithm: {algorithm_name}. "
                     f"Supported: 'qlearning', 'sarsa', 'expected_sarsa', 'double_qlearning'")
