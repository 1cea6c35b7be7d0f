"""Capture-time stub of gymnasium.logger."""
import warnings


def warn(msg, *args, **kwargs):
    warnings.warn(str(msg))
