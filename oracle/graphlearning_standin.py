"""Stand-in for the third-party `graphlearning` package -- TEST INFRASTRUCTURE ONLY.

GLL.py imports `graphlearning as gl` (/root/reference/GLL.py:2) and uses exactly two of its
entry points:

  * `gl.weightmatrix.knnsearch(X, k, similarity='euclidean', method='annoy')`
    (/root/reference/GLL.py:183) -> (knn_ind n x k, knn_dist n x k), nearest first,
    the query point itself first, Euclidean (not squared) distances.
  * `gl.graph(W).gradient(u)` (/root/reference/GLL.py:111-120) -> sparse matrix with
    u[j] - u[i] on the nonzero pattern (i, j) of W (unweighted form).

graphlearning ~=1.6.9 (pinned in /root/reference/requirements.txt:5) and its `annoy`
backend are not installed and not vendored.  annoy is an *approximate* index; this
stand-in is EXACT brute force in float64, which is the documented parity definition
(SURVEY.md §8c): self forced to rank 0 with distance 0, remaining neighbours ordered by
(distance, index).
"""
from __future__ import annotations

import sys
import types

import numpy as np
import scipy.sparse as sparse


def knn_exact(X, k, fast=False):
    """Exact kNN in float64 including self at rank 0. Returns (ind int64, dist float64).

    fast=False: full stable argsort, ties broken by index (fixture semantics).
    fast=True : argpartition + sort of the survivors (timing baseline; ties at the k-th
                boundary may resolve differently, nothing else changes)."""
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[0]
    k = int(min(k, n))
    sq = np.einsum("ij,ij->i", X, X)
    d2 = sq[:, None] + sq[None, :] - 2.0 * (X @ X.T)
    np.maximum(d2, 0.0, out=d2)
    np.fill_diagonal(d2, -1.0)
    if fast and k < n:
        part = np.argpartition(d2, k - 1, axis=1)[:, :k]
        pd = np.take_along_axis(d2, part, axis=1)
        order = np.lexsort((part, pd), axis=1)
        ind = np.take_along_axis(part, order, axis=1)
    else:
        ind = np.argsort(d2, axis=1, kind="stable")[:, :k]
    dist2 = np.take_along_axis(d2, ind, axis=1)
    dist2[:, 0] = 0.0
    return ind.astype(np.int64), np.sqrt(dist2)


class _WeightMatrix:
    fast = False

    def knnsearch(self, X, k, similarity="euclidean", method="annoy"):
        if similarity != "euclidean":
            raise NotImplementedError(similarity)
        return knn_exact(X, k, fast=self.fast)


class _Graph:
    """Pattern-only graph: gradient(u)_{ij} = u_j - u_i on the stored pattern."""

    def __init__(self, W):
        self.I, self.J, _ = sparse.find(W)
        self.n = W.shape[0]

    def gradient(self, u, weighted=False):
        u = np.asarray(u)
        vals = u[self.J] - u[self.I]
        return sparse.coo_matrix((vals, (self.I, self.J)), shape=(self.n, self.n)).tocsr()


def make_module():
    mod = types.ModuleType("graphlearning")
    mod.weightmatrix = _WeightMatrix()
    mod.graph = _Graph
    return mod


def install():
    """Place the stand-in in sys.modules so `import graphlearning` resolves to it."""
    sys.modules["graphlearning"] = make_module()
    return sys.modules["graphlearning"]
