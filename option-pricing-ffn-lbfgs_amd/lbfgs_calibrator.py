"""Drop-in module name of src/calibration/lbfgs_calibrator.py.

``CalibrationResult`` is registered under this module name (dhcos.calibrator sets its
``__module__``), so pickles written here name ``lbfgs_calibrator.CalibrationResult`` exactly as
the reference's do and load on either side (tests/test_suite.py:354-372,
synthetic_generator.py:181-183)."""
from dhcos.calibrator import CalibrationResult, DoubleHestonJumpCalibrator  # noqa: F401

__all__ = ["CalibrationResult", "DoubleHestonJumpCalibrator"]
