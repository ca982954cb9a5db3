"""Portable, bit-reproducible synthetic inputs for the compression path.

Used by the golden generator (tests/golden/gen_golden.py, which feeds the same arrays to the
reference) and by the tests / bench (which feed them to the HIP path and the oracle).  Only integer
arithmetic and correctly-rounded fp32 IEEE operations (+, *, /, a sequential cumsum) are used, so
the arrays are identical on every x86-64 host regardless of SIMD width.

Shapes follow SURVEY.md §8(d): K, V ~ approx. N(0,1); W prompt slice [B,H,S,P] = a peaked,
row-normalised positive distribution scaled by a per-row U(0,1) mass and causal inside the prompt.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n outputs of splitmix64 seeded with (seed, stream)."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x100000001B3 + stream * 0x1000193) & 0xFFFFFFFFFFFFFFFF)
        z = base + (np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, shape, stream: int = 0) -> np.ndarray:
    """U[0,1) with 24-bit resolution as float32 (exact)."""
    n = int(np.prod(shape))
    u = (splitmix64(seed, n, stream) >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    return u.reshape(shape)


def normal(seed: int, shape, stream: int = 0) -> np.ndarray:
    """Irwin-Hall(4) approximation of N(0,1) from the four 16-bit fields of one draw (float32;
    the sum is exact, the final scale is one correctly rounded multiply)."""
    n = int(np.prod(shape))
    x = splitmix64(seed, n, stream)
    m = np.uint64(0xFFFF)
    acc = (x & m).astype(np.float32)
    acc += ((x >> np.uint64(16)) & m).astype(np.float32)
    t = ((x >> np.uint64(32)) & m).astype(np.float32)
    t += (x >> np.uint64(48)).astype(np.float32)
    del x
    acc += t
    acc *= np.float32(2.0 ** -16)
    acc -= np.float32(2.0)
    acc *= np.float32(1.7320508075688772)
    return acc.reshape(shape)


# ----------------------------------------------------------------------------- dtype casting
def to_bf16_bits(x32: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x32, np.float32).view(np.uint32)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + np.uint32(0x7FFF) + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


DTYPES = {"float32": 0, "float16": 1, "bfloat16": 2}


def cast(x: np.ndarray, dtype: str) -> np.ndarray:
    """float32/float64 → dtype storage: float32 array, or uint16 bit patterns for half types."""
    x32 = np.asarray(x).astype(np.float32, copy=False)
    if dtype == "float32":
        return x32
    if dtype == "float16":
        return x32.astype(np.float16).view(np.uint16)
    if dtype == "bfloat16":
        return to_bf16_bits(x32)
    raise ValueError(dtype)


def to_f32(stored: np.ndarray, dtype: str) -> np.ndarray:
    if dtype == "float32":
        return np.asarray(stored, np.float32)
    if dtype == "float16":
        return np.asarray(stored, np.uint16).view(np.float16).astype(np.float32)
    return bf16_bits_to_f32(stored)


# ----------------------------------------------------------------------------- generators
def kv(seed: int, B: int, S: int, F: int, dtype: str, layout: str = "bsf"):
    """K, V storage arrays [B,S,F] (layout 'bsf') from streams 1 and 2 of `seed`."""
    K = cast(normal(seed, (B, S, F), 1), dtype)
    V = cast(normal(seed, (B, S, F), 2), dtype)
    return K, V


def attention_slice(seed: int, B: int, H: int, S: int, P: int, dtype: str, causal: bool = True):
    """W prompt slice [B,H,S,P]: u^4 row-normalised (sequential fp32 cumsum) × U(0,1) row mass."""
    u = uniform(seed, (B, H, S, P), 3)
    raw = u * u
    raw *= raw
    raw += np.float32(1e-6)
    if causal:
        i = np.arange(S)[:, None]
        p = np.arange(P)[None, :]
        raw = np.where(p <= i, raw, np.float32(0.0))
    rs = np.cumsum(raw, axis=-1, dtype=np.float32)[..., -1:]
    m = uniform(seed, (B, H, S, 1), 4)
    W = (raw / rs) * m
    return cast(W, dtype)


def attention_full(seed: int, B: int, H: int, S: int, dtype: str):
    """Full [B,H,S,S] non-causal row-stochastic W (small shapes only, reference test style)."""
    u = uniform(seed, (B, H, S, S), 5)
    raw = u * u + np.float32(1e-3)
    rs = np.cumsum(raw, axis=-1, dtype=np.float32)[..., -1:]
    return cast(raw / rs, dtype)


def scores_like(seed: int, B: int, S: int) -> np.ndarray:
    """float32 importance-like scores in [0, 1] with realistic tie structure."""
    return uniform(seed, (B, S), 6)
