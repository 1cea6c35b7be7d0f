from .advanced import AdvancedForestFireBulldozerEnv
from .batched import BatchedForestFireBulldozerEnv
from .bulldozer import ForestFireBulldozerEnv

__all__ = ["ForestFireBulldozerEnv", "BatchedForestFireBulldozerEnv", "AdvancedForestFireBulldozerEnv"]
