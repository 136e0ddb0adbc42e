"""lietorch on MI355X: SO3 / SE3 groups over the `lietorch_backends` HIP
extension (L-SE3).

API of dpvo/lietorch (cuteboyqq/DPVO: groups.py, group_ops.py,
broadcasting.py): `SE3(data)`, `.inv()`, `*` (group product or action on
points), `.retr(a)`, `.adjT(a)`, `.matrix()`, `.log()`, `SE3.exp(a)`, ...
RxSO3 / Sim3 (group ids 2 and 4) are not on DPVO's per-frame hot path and are
not provided by this build; constructing one raises.
"""
from .groups import LieGroup, LieGroupParameter, RxSO3, SE3, SO3, Sim3, cat, stack  # noqa: F401

__all__ = ["LieGroup", "LieGroupParameter", "SO3", "SE3", "RxSO3", "Sim3", "cat", "stack"]
