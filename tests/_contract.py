"""Operator contract of the reference's tests/test_operator.py:9-67 (assert_operator), restated."""
from gymca_amd.operator import Operator
from gymca_amd.spaces import Space


def assert_operator(op, strict=False):
    def optionals(optional, atts):
        for att in atts:
            v = getattr(op, att)
            assert isinstance(v, optional) or v is None
            if strict:
                assert isinstance(v, optional), f"{att} expected {optional}, got {type(v)}"

    def update():
        grid = op.grid_space.sample()
        action = op.action_space.sample()
        context = op.context_space.sample()
        grid, context = op.update(grid, action, context)
        assert op.grid_space.contains(grid)
        assert op.context_space.contains(context)

    assert isinstance(op, Operator)
    assert isinstance(op.suboperators, tuple)
    for sub in op.suboperators:
        assert_operator(sub)
    optionals(bool, ("grid_dependant", "action_dependant", "context_dependant"))
    optionals(Space, ("grid_space", "action_space", "context_space"))
    optionals(bool, ("deterministic",))
    assert callable(op.update)
    if strict:
        update()
    else:
        try:
            update()
        except AttributeError:
            pass
