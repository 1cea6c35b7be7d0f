"""GPU operators with the reference's names (forest_fire/operators/__init__.py:1-20)."""
from .ca_alexandridis import PartiallyObservableForestFire, PartiallyObservableForestFireJax
from .ca_DrosselSchwabl import ForestFire
from .ca_windy import WindyForestFire
from .move_modify import Modify, Move, MoveModify
from .move_modify_jax import ModifyJax, MoveJax, MoveModifyJax
from .repeat_ca import RepeatCA
from .repeat_ca_jax import RepeatCAJax

__all__ = ["WindyForestFire", "PartiallyObservableForestFire", "PartiallyObservableForestFireJax", "ForestFire",
           "Move", "Modify", "MoveModify", "RepeatCA", "MoveJax", "ModifyJax", "MoveModifyJax", "RepeatCAJax"]
