"""Capture-time stub of gymnasium.error."""


class Error(Exception):
    pass
