"""RL operator interface of the reference (src/model/algorithms.py:10-383).

The classes keep the reference's constructor signature, attributes, eps
schedule (`decay_epsilon`, algorithms.py:40-42) and the `create_algorithm`
factory with its ValueError.

Two execution paths:
  * `SPGG.run` / `BatchEngine` never call these methods: the per-lattice
    `select_action` / `update_q_table` arithmetic of the four operators is fused into
    the HIP step (libspgg_hip.so, one template instance per operator);
  * a caller that uses the operator interface directly (the reference's own
    `algorithm.select_action(...)` / `.update_q_table(...)` calls, spgg.py:410-441)
    gets the same results on the host: the methods below are NumPy restatements that
    consume the global `np.random` stream exactly as the reference's do (rand, then
    randint per select; Double-Q's rand < 0.5 table choice), so a mixed host / device
    caller keeps the reference's stream.  Pinned bit for bit by
    tests/golden/operator_calls.npz (made by importing the reference,
    tests/golden/make_operator_golden.py; tests/test_operator_host_cpu.py).

The plug-in point (`SPGG(algorithm=<RLAlgorithm instance>)`, spgg.py:111-118):
`operator_kind` accepts these four classes, the reference's own four (an
instance built from src/model/algorithms.py drops in) and subclasses that only
add state; anything that redefines the operator's methods is refused with a
ValueError naming the class, so custom arithmetic can never silently run as the
built-in operator.
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
        """eps-greedy actions over the (L, L) lattice (algorithms.py:102-110, the same in all
        four operators): ONE rand(L, L) then ONE randint(0, 2, (L, L)) from the global stream;
        greedy = first argmax of the agent's row Q[i, j, s_ij, :] (ties -> action 0)."""
        return _eps_greedy(q_table, states, L, self.epsilon)

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        """TD update of entry (s, a) of every agent, in place; returns the table."""
        raise NotImplementedError("RLAlgorithm.update_q_table is abstract (algorithms.py:44-70)")

    def _td(self, q_table, old_states, actions, rewards, target):
        """Q[s, a] <- Q[s, a] + alpha * ((r + gamma * target) - Q[s, a]) in place: the
        reference's evaluation order (algorithms.py:128-131)."""
        q = _entries(q_table, old_states, actions)
        td = rewards + self.gamma * target - q
        _put_entries(q_table, old_states, actions, q + self.alpha * td)
        return q_table


def _rows(q_table, states):
    """Q[i, j, states[i, j], :] of every agent, shape (L, L, actions)."""
    s = np.asarray(states)
    return np.take_along_axis(q_table, s[:, :, None, None], axis=2)[:, :, 0, :]


def _entries(q_table, states, actions):
    """Q[i, j, states[i, j], actions[i, j]], shape (L, L)."""
    row = _rows(q_table, states)
    return np.take_along_axis(row, np.asarray(actions)[:, :, None], axis=2)[:, :, 0]


def _put_entries(q_table, states, actions, values):
    """Q[i, j, states[i, j], actions[i, j]] = values (each agent's entry written once)."""
    L0, L1 = q_table.shape[:2]
    ii, jj = np.meshgrid(np.arange(L0), np.arange(L1), indexing="ij")
    q_table[ii, jj, np.asarray(states), np.asarray(actions)] = values


def _eps_greedy(q_table, states, L, epsilon):
    """algorithms.py:105-109: explore = rand < eps (drawn first), greedy = argmax of the row
    (first maximum), random action = randint(0, 2) (drawn second)."""
    explore = np.random.rand(L, L) < epsilon
    greedy = np.argmax(_rows(q_table, states), axis=2)
    random_action = np.random.randint(0, 2, size=(L, L))
    return np.where(explore, random_action, greedy)


class QLearning(RLAlgorithm):
    """Off-policy TD with max over next-state actions (algorithms.py:96-133)."""
    kind = "qlearning"

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        """target = max_a' Q[s', a'] (algorithms.py:124-131)."""
        return self._td(q_table, old_states, actions, rewards, _rows(q_table, new_states).max(axis=2))


class SARSA(RLAlgorithm):
    """On-policy TD (algorithms.py:136-178)."""
    kind = "sarsa"

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        """target = Q[s', a'] of the next actions the caller passes (algorithms.py:159-176)."""
        if "next_actions" not in kwargs:
            raise ValueError("SARSA requires 'next_actions' parameter")
        target = _entries(q_table, new_states, kwargs["next_actions"])
        return self._td(q_table, old_states, actions, rewards, target)


class ExpectedSARSA(RLAlgorithm):
    """Expected-value TD under the eps-greedy policy (algorithms.py:181-234)."""
    kind = "expected_sarsa"

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        """target = sum_a' pi(a'|s') Q[s', a'] with pi eps-greedy: eps / A everywhere plus
        (1 - eps) on the first argmax, summed over a' in order (algorithms.py:212-229)."""
        nxt = _rows(q_table, new_states)
        A = q_table.shape[3]
        other = self.epsilon / A
        probs = np.full(nxt.shape, other)
        greedy = np.argmax(nxt, axis=2)
        np.put_along_axis(probs, greedy[:, :, None], (1 - self.epsilon) + other, axis=2)
        return self._td(q_table, old_states, actions, rewards, np.sum(probs * nxt, axis=2))


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

    def select_action(self, q_table, states, L, **kwargs):
        """eps-greedy on the mean table; before initialize_q_tables on the table passed in
        (algorithms.py:268-290)."""
        if self.q_table_1 is None or self.q_table_2 is None:
            return _eps_greedy(q_table, states, L, self.epsilon)
        return _eps_greedy(self.get_combined_q_table(), states, L, self.epsilon)

    def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
        """Per agent one rand(L, L) < 0.5 picks the table updated (q_table_1 where true),
        evaluated at the OTHER table's greedy next action; returns the mean table
        (algorithms.py:292-341; the q_table argument is not read)."""
        if self.q_table_1 is None or self.q_table_2 is None:
            raise ValueError("Q-tables not initialized. Call initialize_q_tables first.")
        L = self.q_table_1.shape[0]
        first = np.random.rand(L, L) < 0.5
        n1, n2 = _rows(self.q_table_1, new_states), _rows(self.q_table_2, new_states)
        # Q1's target: Q2 at Q2's argmax; Q2's target: Q1 at Q1's argmax (= each row's max)
        t1, t2 = n2.max(axis=2), n1.max(axis=2)
        for tab, target, mask in ((self.q_table_1, t1, first), (self.q_table_2, t2, ~first)):
            q = _entries(tab, old_states, actions)
            new = q + self.alpha * (rewards + self.gamma * target - q)
            _put_entries(tab, old_states, actions, np.where(mask, new, q))
        return self.get_combined_q_table()


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
