"""Drop-in module name of src/data/synthetic_generator.py."""
from dhcos.generator import generate_synthetic_calibrations  # noqa: F401

__all__ = ["generate_synthetic_calibrations"]
