"""numpy mirror of wx_fill_synthetic (include/warpexec.h) for host-side checks.

h = splitmix64(row + seed * 0xD1B54A32D192ED03)
  kind 0 (uniform float): lo + ((h >> 40) * 2^-24) * (hi - lo), in float32
  kind 1 (uniform int):   lo + (h >> 32) % (hi - lo + 1)
"""
from __future__ import annotations

import numpy as np

_M = np.uint64


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + _M(0x9E3779B97F4A7C15)
        x = (x ^ (x >> _M(30))) * _M(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> _M(27))) * _M(0x94D049BB133111EB)
        return x ^ (x >> _M(31))


def _hash(n: int, seed: int, row_base: int = 0) -> np.ndarray:
    rows = np.arange(row_base, row_base + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64(rows + _M(seed) * _M(0xD1B54A32D192ED03))


def uniform_f32(n: int, seed: int, lo: float, hi: float, row_base: int = 0) -> np.ndarray:
    h = _hash(n, seed, row_base)
    u = (h >> _M(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    span = np.float32(hi) - np.float32(lo)
    return (np.float32(lo) + u * span).astype(np.float32)


def uniform_int(n: int, seed: int, lo: int, hi: int, row_base: int = 0) -> np.ndarray:
    h = _hash(n, seed, row_base)
    return (np.int64(lo) + ((h >> _M(32)) % _M(hi - lo + 1)).astype(np.int64))


# The bench / BASELINE.json tables
SEED_PRICE, SEED_QTY, SEED_KEY = 1, 2, 3


def c2_table(n: int, row_base: int = 0):
    """price f32 U[0,40), quantity f32 integer-valued U{1..100}."""
    return {
        "price": uniform_f32(n, SEED_PRICE, 0.0, 40.0, row_base),
        "quantity": uniform_int(n, SEED_QTY, 1, 100, row_base).astype(np.float32),
    }


def c3_table(n: int, row_base: int = 0):
    """price f32 U[0,40), quantity int32 U{0..1023} (1K groups)."""
    return {
        "price": uniform_f32(n, SEED_PRICE, 0.0, 40.0, row_base),
        "quantity": uniform_int(n, SEED_KEY, 0, 1023, row_base).astype(np.int32),
    }
