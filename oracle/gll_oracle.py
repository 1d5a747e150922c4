"""Float64 closed-form restatement of LaplaceLearningSparseHard -- TEST INFRASTRUCTURE ONLY.

This is the parity checker for the HIP path.  It restates /root/reference/GLL.py in closed
form and is pinned against fixtures produced by the reference module itself
(tests/golden/, tests/test_oracle_golden.py).  Never imported by the product package.

Closed form (n = base + m rows, labeled rows first; K = neighbours incl. self):
  E     = union of directed kNN pairs, self and zero-distance pairs dropped   GLL.py:192-198
  eps_i = eps (fixed, GLL.py:226) | d(i, knn_ind[i, K-1]) (auto, GLL.py:205)
  W_ij  = exp(-4 d_ij^2 / (eps_i eps_j))                                      GLL.py:216/233
  L     = diag(rowsum W) - W ; Luu = L[base:, base:] + tau I ; Lul = L[base:, :base]
  U     = Luu^{-1} (-Lul Y)                                                    GLL.py:29-53
  wU    = Luu^{-1} gbar ; w = [0; wU] ; P = [Y; U]                             GLL.py:93-109
  G_ij  = sum_c (w_ic - w_jc)(P_jc - P_ic)                                     GLL.py:111-120
  V_ij  = -8 W_ij / (eps_i eps_j) ; S_ij = G_ij V_ij                           GLL.py:217,146
  grad_i = sum_j S_ij (x_i - x_j)                                              GLL.py:148-159
     [auto] - b_i (x_i - x_kth(i)) - sum_{l: kth(l)=i} b_l (x_i - x_l),
            b_i = sum_j G_ij d_ij^2 V_ij / (2 eps_i^2)                         GLL.py:124-139
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sparse
import scipy.sparse.linalg as spla

from .graphlearning_standin import knn_exact


@dataclass
class Graph:
    n: int
    rows: np.ndarray      # int64 E, sorted by (row, col)
    cols: np.ndarray      # int64 E
    dist: np.ndarray      # float64 E, Euclidean distance
    eps: np.ndarray       # float64 n
    kth: np.ndarray       # int64 n (knn_ind[:, K-1])
    auto: bool

    @property
    def W(self) -> np.ndarray:
        return np.exp(-4.0 * self.dist ** 2 / (self.eps[self.rows] * self.eps[self.cols]))

    def csr(self, vals) -> sparse.csr_matrix:
        return sparse.csr_matrix((vals, (self.rows, self.cols)), shape=(self.n, self.n))


def graph_from_knn(knn_ind, knn_dist, epsilon) -> Graph:
    """Symmetrised kNN graph; restates knn_sym_dist (GLL.py:180-244)."""
    knn_ind = np.asarray(knn_ind, dtype=np.int64)
    knn_dist = np.asarray(knn_dist, dtype=np.float64)
    n, K = knn_ind.shape
    r = np.repeat(np.arange(n), K)
    D = sparse.coo_matrix((knn_dist.ravel(), (r, knn_ind.ravel())), shape=(n, n)).tocsr()
    D = D.maximum(D.T)                       # union pattern, max of the two directions
    rows, cols, vals = sparse.find(D)        # drops self (0) and zero distances
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    kth = knn_ind[:, K - 1]
    auto = isinstance(epsilon, str)
    if auto:
        if epsilon != "auto":
            raise ValueError(epsilon)
        eps = np.asarray(D[np.arange(n), kth]).ravel()
    else:
        eps = float(epsilon) * np.ones(n)
    if (eps < 1e-10).any():
        warnings.warn("Epsilon in KNN is very close to zero.", UserWarning)
    return Graph(n, rows.astype(np.int64), cols.astype(np.int64), vals, eps, kth, auto)


@dataclass
class State:
    X: np.ndarray
    Y: np.ndarray
    U: np.ndarray
    tau: float
    graph: Graph
    Luu: sparse.csr_matrix


def forward(X, Y, tau=0.0, epsilon="auto", K=25, knn=None):
    """Return (U m x C float64, State).  `knn` = (ind, dist) overrides the exact search."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    base = Y.shape[0]
    n = X.shape[0]
    if knn is None:
        ind, dist = knn_exact(X, K)
    else:
        ind = np.asarray(knn[0], dtype=np.int64)
        if knn[1] is not None:
            dist = np.asarray(knn[1], dtype=np.float64)
        else:  # exact float64 distances of the given pairs, row blocks to bound memory
            dist = np.empty(ind.shape)
            for r0 in range(0, n, 256):
                blk = ind[r0:r0 + 256]
                dist[r0:r0 + 256] = np.sqrt(np.sum(
                    (X[r0:r0 + 256, None, :] - X[blk]) ** 2, axis=2))
    g = graph_from_knn(ind, dist, epsilon)
    W = g.csr(g.W)
    deg = np.asarray(W.sum(axis=1)).ravel()
    L = (sparse.diags(deg) - W).tocsr()
    m = n - base
    Luu = (L[base:, base:] + float(tau) * sparse.identity(m, format="csr")).tocsc()
    rhs = -(L[base:, :base] @ Y)
    U = np.asarray(spla.spsolve(Luu, rhs)).reshape(m, -1)
    return U, State(X, Y, U, float(tau), g, Luu)


def edge_coefficients(state: State, gbar):
    """Per-edge S_ij (plus folded auto terms) and b; the quantities backward needs."""
    g = state.graph
    base = state.Y.shape[0]
    gbar = np.asarray(gbar, dtype=np.float64).reshape(state.U.shape)
    wU = np.asarray(spla.spsolve(state.Luu, gbar)).reshape(state.U.shape)
    w = np.concatenate([np.zeros_like(state.Y), wU], axis=0)
    P = np.concatenate([state.Y, state.U], axis=0)
    r, c = g.rows, g.cols
    G = np.sum((w[r] - w[c]) * (P[c] - P[r]), axis=1)
    V = -8.0 * g.W / (g.eps[r] * g.eps[c])
    S = G * V
    b = None
    if g.auto:
        modV = g.dist ** 2 * V / (2.0 * g.eps[r] ** 2)
        b = np.bincount(r, weights=G * modV, minlength=g.n)
        coef = S.copy()
        coef -= np.where(c == g.kth[r], b[r], 0.0)
        coef -= np.where(g.kth[c] == r, b[c], 0.0)
    else:
        coef = S
    return coef, b, wU


def backward(state: State, gbar):
    """grad_X (n x d float64) for upstream gradient gbar (m x C)."""
    coef, _, _ = edge_coefficients(state, gbar)
    g = state.graph
    Sm = g.csr(coef)
    rowsum = np.asarray(Sm.sum(axis=1)).ravel()
    return rowsum[:, None] * state.X - Sm @ state.X


def knn_set_mismatch(X, ind_test, K, rel_gap=1e-5):
    """Rows whose kNN set differs from the exact float64 set beyond near-ties.

    A row is excused when the exact squared distances of the swapped-in and swapped-out
    neighbours differ by less than `rel_gap` relative (SURVEY.md §8c kNN rule)."""
    X = np.asarray(X, dtype=np.float64)
    ind_ref, dist_ref = knn_exact(X, K)
    bad = []
    for i in range(X.shape[0]):
        a, b = set(ind_ref[i].tolist()), set(np.asarray(ind_test[i]).tolist())
        if a == b:
            continue
        kth2 = dist_ref[i, -1] ** 2
        extra = np.array(sorted(b - a))
        d2 = np.sum((X[extra] - X[i]) ** 2, axis=1) if extra.size else np.zeros(0)
        if extra.size == 0 or np.any(np.abs(d2 - kth2) > rel_gap * max(kth2, 1e-30)):
            bad.append(i)
    return bad


def rel_err(a, b) -> float:
    """||a - b||_inf / ||b||_inf (the parity metric of SURVEY.md §8c)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.max(np.abs(b))
    return float(np.max(np.abs(a - b)) / (den if den > 0 else 1.0))


# ----------------------------------------------------------------------------------------
# utils.laplace: the large single-graph evaluation path
# ----------------------------------------------------------------------------------------
def one_hot_encode(labels, n_classes="auto"):
    """utils.py:556-568: labels -> n_labels x C one-hot, C = #unique labels when 'auto'."""
    labels = np.asarray(labels)
    C = len(np.unique(labels)) if n_classes == "auto" else int(n_classes)
    Y = np.zeros((len(labels), C))
    Y[np.arange(len(labels)), labels] = 1
    return Y


def laplace(X, train_labels, knn_num=50, epsilon="auto", n_classes="auto", tau=1e-8, knn=None):
    """utils.py:570-593 in closed form: W from the symmetrised kNN graph (knn_sym_dist), L =
    D - W (csgraph.laplacian, utils.py:575), Luu = L[k:,k:] + tau I, rhs = -Lul Y; the
    reference solves the Jacobi-scaled system (M Luu M) y = M rhs with stable_conjgrad to
    1e-10 and returns M y (utils.py:585-592) -- mathematically Luu^{-1} rhs, solved here
    directly (SuperLU).  `knn` = (ind, dist) overrides the exact search."""
    X = np.asarray(X, dtype=np.float64)
    Y = one_hot_encode(train_labels, n_classes)
    k = Y.shape[0]
    if knn is None:
        ind, dist = knn_exact(X, knn_num)
    else:
        ind, dist = knn
        if dist is None:
            dist = np.sqrt(((X[:, None, :] - X[np.asarray(ind)]) ** 2).sum(-1))
    g = graph_from_knn(ind, dist, epsilon)
    W = g.csr(g.W)
    deg = np.asarray(W.sum(axis=0)).ravel()
    L = (sparse.diags(deg) - W).tocsr()
    m = g.n - k
    Luu = (L[k:, k:] + tau * sparse.eye(m)).tocsc()
    rhs = -(L[k:, :k] @ Y)
    return spla.spsolve(Luu, rhs).reshape(m, -1)
