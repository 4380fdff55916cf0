"""Drop-in module name of src/models/double_heston.py: ``from double_heston import DoubleHeston``
resolves to the gfx950-backed class (dhcos.pricer)."""
from dhcos.pricer import DoubleHeston  # noqa: F401

__all__ = ["DoubleHeston"]
