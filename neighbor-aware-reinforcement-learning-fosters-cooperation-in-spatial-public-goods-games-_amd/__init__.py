"""spgg_amd — MI355X-native hot path of the neighbor-aware RL Spatial Public Goods Game.

Drop-in for the reference's `src.model` (SPGG + RL operator interface), with
the per-iteration step (src/model/spgg.py:368-592) executed by hand-written
HIP kernels for gfx950 in libspgg_hip.so (C ABI: include/spgg_abi.h).
"""
from .algorithms import (RLAlgorithm, QLearning, SARSA, ExpectedSARSA,  # noqa: F401
                         DoubleQLearning, create_algorithm)
from .engine import BatchEngine, InitState, ReplicaParams, reference_init  # noqa: F401
from .spgg import SPGG, sum_position_and_neighbors, cluster_sizes  # noqa: F401

__all__ = ['SPGG', 'RLAlgorithm', 'QLearning', 'SARSA', 'ExpectedSARSA',
           'DoubleQLearning', 'create_algorithm', 'BatchEngine', 'ReplicaParams',
           'InitState', 'reference_init']
__version__ = "0.1.0"
