"""Synthetic minibatch features for the GLL hot path (SURVEY.md §8d generator).

The reference feeds `LaplaceLearningSparseHard` with unit-norm encoder features
(`F.normalize` at /root/reference/networks/BuildNet.py:101) whose labeled rows come first
(/root/reference/FullySup.py:153-154).  iid Gaussians make a useless graph (SURVEY.md §0
item 9), so this draws a latent class mixture lifted into d dimensions:

    centre_c ~ r * N(0, I_latent)                      per class c
    z_i      = centre_{label_i} + N(0, I_latent)       label_i = i mod C
    X_i      = normalize(Q z_i + iso * N(0, I_d))       Q: d x latent orthonormal

Everything is built from numpy's PCG64 stream and single IEEE elementwise operations
(no BLAS, no LAPACK), so the float32 matrix is bit-identical on any x86 host that runs
this image.  `sha256(X)` is stored next to the golden fixtures to check that.
"""
from __future__ import annotations

import hashlib

import numpy as np

# Named configs of BASELINE.json (configs[0..4]); r = centre spread.
CONFIGS = {
    "plumbing": dict(base=64, batch=64, d=32, k=5, r=0.75),
    "ns": dict(base=500, batch=500, d=512, k=10, r=1.0),
    "fullysup": dict(base=250, batch=1250, d=128, k=25, r=1.0),
    "stress": dict(base=4096, batch=4096, d=1024, k=30, r=1.0),
}


def _orthonormal_columns(g: np.ndarray) -> np.ndarray:
    """Modified Gram-Schmidt with elementwise ufuncs only (bit-reproducible)."""
    q = np.empty_like(g)
    for k in range(g.shape[1]):
        v = g[:, k].copy()
        for j in range(k):
            v = v - np.sum(q[:, j] * v) * q[:, j]
        q[:, k] = v / np.sqrt(np.sum(v * v))
    return q


def synth(base: int, batch: int, d: int, C: int = 10, r: float = 1.0, latent: int = 16,
          iso: float = 0.05, seed: int = 0):
    """Return (X float32 n x d unit rows, labels int64 n) with labeled rows first."""
    n = base + batch
    rng = np.random.Generator(np.random.PCG64(seed))
    centres = r * rng.standard_normal((C, latent))
    labels = np.arange(n, dtype=np.int64) % C
    z = centres[labels] + rng.standard_normal((n, latent))
    q = _orthonormal_columns(rng.standard_normal((d, latent)))
    x = iso * rng.standard_normal((n, d))
    for k in range(latent):
        x = x + z[:, k:k + 1] * q[:, k][None, :]
    x = x / np.sqrt(np.sum(x * x, axis=1, keepdims=True))
    return x.astype(np.float32), labels


def one_hot(labels: np.ndarray, C: int = 10) -> np.ndarray:
    out = np.zeros((labels.shape[0], C), dtype=np.float32)
    out[np.arange(labels.shape[0]), labels] = 1.0
    return out


def seeded_gbar(m: int, C: int, seed: int = 1234) -> np.ndarray:
    """Fixed upstream gradient dL/dU (m x C float64) used instead of a loss in parity tests."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal((m, C))


def sha256(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
