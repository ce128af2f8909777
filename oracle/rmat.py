"""Counter-based Graph500 R-MAT generator, numpy twin (TEST INFRASTRUCTURE ONLY).

The reference generates benchmark inputs with RAFT's RNG
(``cpp/src/generators/generate_rmat_edgelist.cu:36-103``, parameters from
``benchmarks/python_e2e/cugraph_funcs.py:40-60``: a=0.57, b=c=0.19, edge factor
16, seed 42, ``clip_and_flip=False``, ``scramble_vertex_ids=True``).  RAFT is not
available here, so graph identity with the reference is "parity unpinned" (as
the reference's own RMAT tests, we compare GPU vs CPU on the *same* generated
graph).  This module defines the generator; ``cugraph-forked_amd/csrc/rmat.hip``
must produce bit-identical edges (``tests/test_rmat.py`` checks it).

Definition (per edge e, per level l = 0..scale-1, most significant bit first):
  x  = seed * 0x9E3779B97F4A7C15 ^ (e * 64 + l)          (mod 2^64)
  z  = splitmix64(x)
  r  = (z >> 11) * 2^-53                                  (double in [0,1))
  r < a: (0,0);  r < a+b: (0,1);  r < a+b+c: (1,0);  else (1,1)   -> (src bit, dst bit)
Scramble (bijective on [0, 2^scale)):  v = (v*0x9E3779B1 + seed) & mask;
  v ^= v >> h;  v = (v*0x85EBCA77) & mask;  v ^= v >> h   with h = (scale+1)//2.
Weights: w_e = (splitmix64(seed2 * 0x9E3779B97F4A7C15 ^ e) >> 40) * 2^-24  (exact fp32).
"""
from __future__ import annotations

import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _u01(seed: int, e: np.ndarray, level: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * _G) ^ (e * np.uint64(64) + np.uint64(level))
    z = splitmix64(x)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def scramble(v: np.ndarray, scale: int, seed: int) -> np.ndarray:
    v = np.asarray(v, dtype=np.uint64)
    if scale == 0:
        return v
    mask = np.uint64((1 << scale) - 1)
    h = np.uint64((scale + 1) // 2)
    with np.errstate(over="ignore"):
        v = (v * np.uint64(0x9E3779B1) + np.uint64(seed)) & mask
        v = v ^ (v >> h)
        v = (v * np.uint64(0x85EBCA77)) & mask
        v = v ^ (v >> h)
    return v


def rmat(scale, num_edges, a=0.57, b=0.19, c=0.19, seed=42, clip_and_flip=False,
         scramble_vertex_ids=True, first_edge=0, chunk=1 << 22):
    """Edges [first_edge, first_edge+num_edges) of the stream; returns int64 (src, dst)."""
    tab = a + b
    tabc = a + b + c
    src = np.zeros(num_edges, dtype=np.uint64)
    dst = np.zeros(num_edges, dtype=np.uint64)
    for lo in range(0, num_edges, chunk):
        hi = min(num_edges, lo + chunk)
        e = np.arange(first_edge + lo, first_edge + hi, dtype=np.uint64)
        s = np.zeros(hi - lo, dtype=np.uint64)
        d = np.zeros(hi - lo, dtype=np.uint64)
        for level in range(scale):
            r = _u01(seed, e, level)
            sb = (r >= tab).astype(np.uint64)
            db = (((r >= a) & (r < tab)) | (r >= tabc)).astype(np.uint64)
            bit = np.uint64(scale - 1 - level)
            s |= sb << bit
            d |= db << bit
        if clip_and_flip:
            swap = s < d
            s2 = np.where(swap, d, s)
            d = np.where(swap, s, d)
            s = s2
        if scramble_vertex_ids:
            s = scramble(s, scale, seed)
            d = scramble(d, scale, seed)
        src[lo:hi] = s
        dst[lo:hi] = d
    return src.astype(np.int64), dst.astype(np.int64)


def rmat_weights(num_edges, seed=42, first_edge=0):
    """Uniform [0,1) fp32 edge weights (24-bit, exactly representable)."""
    e = np.arange(first_edge, first_edge + num_edges, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) * _G) ^ e
    z = splitmix64(x)
    return ((z >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)).astype(np.float32)
