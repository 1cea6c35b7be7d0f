from .helicopter import ForestFireHelicopterEnv

__all__ = ["ForestFireHelicopterEnv"]
