"""CPU check of the erf approximation the 16-bit engines' GELU uses (csrc/irx_common.h erf_as: Abramowitz &
Stegun 7.1.26), restated in float32 numpy: |erf_as - erf| <= 1e-6 over [-8, 8] (stated bound 1.5e-7; fp32
cancellation near 0 adds 5e-7), and the GELU built on it within 1e-6 relative of the exact-erf GELU (a bf16 rounding is 3.9e-3)."""
import numpy as np
from scipy.special import erf


def erf_as(x):
    x = x.astype(np.float32)
    ax = np.abs(x)
    t = (np.float32(1) / (np.float32(0.3275911) * ax + np.float32(1))).astype(np.float32)
    p = np.float32(1.061405429) * t + np.float32(-1.453152027)
    p = p * t + np.float32(1.421413741)
    p = p * t + np.float32(-0.284496736)
    p = p * t + np.float32(0.254829592)
    p = (p * t).astype(np.float32)
    r = (np.float32(1) - p * np.exp(-ax * ax).astype(np.float32)).astype(np.float32)
    return np.copysign(r, x)


def test_erf_as_accuracy():
    x = np.linspace(-8, 8, 2_000_001, dtype=np.float32)
    err = np.abs(erf_as(x).astype(np.float64) - erf(x.astype(np.float64)))
    assert err.max() <= 1e-6, err.max()   # (6.1e-7 near 0: the 1 - p e cancellation in fp32)


def test_gelu_erf_as():
    g = np.linspace(-12, 12, 400_001, dtype=np.float32)
    exact = 0.5 * g.astype(np.float64) * (1 + erf(g.astype(np.float64) / np.sqrt(2)))
    h = np.float32(0.5) * g
    fast = h * erf_as(g * np.float32(0.70710678118654752)) + h
    assert np.max(np.abs(fast - exact)) <= 2e-6 * np.maximum(1, np.abs(g)).max()
