"""gymca_amd — MI355X-native forest-fire cellular-automaton environments.

Drop-in for gym-cellular-automata's Operator / CAEnv API (reference operator.py,
ca_env.py) with every CA step, Move/Modify and reward/done count computed by
hand-written HIP kernels for gfx950 (libgca_hip.so, C-ABI in include/gca.h).
"""
from ._lib import GCAError, load
from .ca_env import CAEnv
from .grid_space import GridSpace
from .operator import Operator

__version__ = "0.1.0"

envs = ["ForestFireHelicopter5x5-v1", "ForestFireBulldozer256x256-v4"]
prototypes = ["ForestFireHelicopterEnv", "ForestFireBulldozerEnv", "AdvancedForestFireBulldozerEnv"]

__all__ = ["GCAError", "load", "CAEnv", "GridSpace", "Operator", "envs", "prototypes"]
