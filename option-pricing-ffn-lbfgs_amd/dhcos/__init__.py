"""dhcos -- MI355X-native Double-Heston + Merton-jump COS pricing and calibration.

Drop-in host API for the hot path of zenthepen/Option-Pricing-FFN-LBFGS:

    DoubleHeston                      src/models/double_heston.py
    DoubleHestonJumpCalibrator,       src/calibration/lbfgs_calibrator.py
    CalibrationResult
    generate_synthetic_calibrations   src/data/synthetic_generator.py

All pricing arithmetic runs in libdhcos.so (hand-written gfx950 HIP kernels, C-ABI in
include/dhcos.h); the native library is loaded on first use and there is no CPU fallback.
The reference's module names (double_heston, lbfgs_calibrator, synthetic_generator) sit next to
this package as one-line re-exports, and ``dhcos.distributed`` (import it explicitly; it needs
torch) shards starts / samples over ``torch.distributed`` ranks (one process per GPU).
"""
from .pricer import DoubleHeston
from .calibrator import CalibrationResult, DoubleHestonJumpCalibrator
from .generator import generate_synthetic_calibrations
from ._native import NativeError

__all__ = ["DoubleHeston", "DoubleHestonJumpCalibrator", "CalibrationResult",
           "generate_synthetic_calibrations", "NativeError"]
__version__ = "0.1.0"
