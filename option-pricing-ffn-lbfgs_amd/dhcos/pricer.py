"""Drop-in ``DoubleHeston`` whose arithmetic runs in the gfx950 kernels of libdhcos.so.

Mirrors the public surface of the reference class (src/models/double_heston.py:8-192):
same constructor signature and attributes, ``pricing(N=128)`` returning an ``np.float64``,
and ``characteristic_function`` / ``truncationRange`` / ``chi_k`` / ``psi_k`` still callable.
Every one of them is evaluated on the GPU through the C-ABI (include/dhcos.h); nothing here
computes a price on the CPU.  ``price_batch`` is the new batched entry point (one launch for any
number of (param set, option) pairs).
"""
from __future__ import annotations

import numpy as np

from . import _native

# constructor order of the 13 model parameters (double_heston.py:26-27)
MODEL_FIELDS = ("v01", "kappa1", "theta1", "sigma1", "rho1", "v02", "kappa2", "theta2",
                "sigma2", "rho2", "lambda_j", "mu_j", "sigma_j")


def resolve_call(option_type) -> bool:
    """Reference rule (double_heston.py:172): call iff option_type.upper()[0] == 'C'.
    Anything else is a put; '' raises IndexError exactly like the reference."""
    return option_type.upper()[0] == "C"


def param_record(model13, S0, r, q=0.0) -> np.ndarray:
    """Pack one DH_PARAM_STRIDE record: 13 model params, S0, r, q."""
    rec = np.empty(_native.PARAM_STRIDE)
    rec[:13] = model13
    rec[13], rec[14], rec[15] = S0, r, q
    return rec


class DoubleHeston:
    """Double Heston + lognormal (Merton) jumps, European call/put by the COS method."""

    def __init__(self, S0, K, T, r, v01, kappa1, theta1, sigma1, rho1,
                 v02, kappa2, theta2, sigma2, rho2, lambda_j, mu_j, sigma_j, option_type="C",
                 q=0.0, *, device=None):
        self.S0, self.K, self.T, self.r, self.q = S0, K, T, r, q
        self.v01, self.kappa1, self.theta1, self.sigma1, self.rho1 = v01, kappa1, theta1, sigma1, rho1
        self.v02, self.kappa2, self.theta2, self.sigma2, self.rho2 = v02, kappa2, theta2, sigma2, rho2
        self.option_type = option_type
        self.lambda_j, self.mu_j, self.sigma_j = lambda_j, mu_j, sigma_j
        self.device = device

    # -- helpers --------------------------------------------------------------------------
    def _ctx(self):
        return _native.default_context(self.device)

    def _record(self) -> np.ndarray:
        return param_record([getattr(self, f) for f in MODEL_FIELDS], self.S0, self.r, self.q)

    # -- reference API --------------------------------------------------------------------
    def characteristic_function(self, phi, tau):
        """phi(u; tau) for real or complex ``phi`` (scalar or array) -- double_heston.py:48-97.
        Real input takes the real-frequency kernel; complex input (any complex dtype, even with
        a zero imaginary part) the complex-frequency one, as the reference's complex arithmetic."""
        u = np.asarray(phi)
        if np.iscomplexobj(u):
            vals = self._ctx().cf_complex(self._record(), u.reshape(-1), tau)
        elif u.dtype.kind in "biuf":
            vals = self._ctx().cf(self._record(), u.astype(np.float64).reshape(-1), tau)
        else:
            raise TypeError(f"phi must be real or complex, got dtype {u.dtype}")
        return vals.reshape(u.shape) if u.ndim else np.complex128(vals[0])

    def truncationRange(self, L=10):
        """(a, b) -- double_heston.py:100-139 (c1 double-counts r*T, log-strike clamp)."""
        a, b = self._ctx().trunc_range(self._record()[None, :], [self.K], [self.T], L)
        return np.float64(a[0]), np.float64(b[0])

    def chi_k(self, k, c, d, a, b):
        """Cosine coefficient of e^y on [c, d] -- double_heston.py:141-151."""
        chi, _ = self._ctx().cos_coeffs([int(k)], c, d, a, b)
        return np.float64(chi[0])

    def psi_k(self, k, c, d, a, b):
        """Cosine coefficient of 1 on [c, d] -- double_heston.py:153-158."""
        _, psi = self._ctx().cos_coeffs([int(k)], c, d, a, b)
        return np.float64(psi[0])

    def pricing(self, N=128):
        """COS price with N terms -- double_heston.py:160-192."""
        is_call = resolve_call(self.option_type)
        return np.float64(self._ctx().price_one(self._record(), float(self.K), float(self.T),
                                                is_call, N))

    # -- batched entry point ----------------------------------------------------------------
    @staticmethod
    def price_batch(params, S0, K, T, r, option_type="C", N=128, q=0.0, L=10.0, device=None):
        """Price option i under param set i, all in one launch.

        params: [n, 13] model parameters (constructor order); S0, K, T, r, q broadcast to n;
        option_type: a string or a sequence of n strings (reference rule) or booleans (is_call).
        """
        params = np.atleast_2d(np.asarray(params, dtype=np.float64))
        n = max(params.shape[0], np.size(K), np.size(T), np.size(S0))
        P = np.broadcast_to(params, (n, 13))
        rec = np.empty((n, _native.PARAM_STRIDE))
        rec[:, :13] = P
        rec[:, 13] = np.broadcast_to(np.asarray(S0, dtype=np.float64), (n,))
        rec[:, 14] = np.broadcast_to(np.asarray(r, dtype=np.float64), (n,))
        rec[:, 15] = np.broadcast_to(np.asarray(q, dtype=np.float64), (n,))
        if isinstance(option_type, str):
            ic = np.full(n, resolve_call(option_type))
        else:
            ot = list(option_type)
            ic = np.array([resolve_call(o) if isinstance(o, str) else bool(o) for o in ot])
            ic = np.broadcast_to(ic, (n,))
        Kb = np.broadcast_to(np.asarray(K, dtype=np.float64), (n,))
        Tb = np.broadcast_to(np.asarray(T, dtype=np.float64), (n,))
        return _native.default_context(device).price_pairs(rec, Kb, Tb, ic, N, L)
