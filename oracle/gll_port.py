"""The reference's CPU step sequence, for the CPU baseline -- TEST INFRASTRUCTURE ONLY.

`bench.py`'s `cpu_baseline` leg times this ("kind": "port") on the GPU box's host cores,
because /root/reference may not travel there.  It performs the same library work, in the
same order, as /root/reference/GLL.py -- exact GEMM kNN (stand-in for annoy), scipy COO/CSR
symmetrisation, `csgraph.laplacian`, SuperLU `spsolve` for the forward and adjoint solves,
the per-class sparse gradient loop, the auto-eps Laplacian term and torch sparse-COO @ X --
so its cost tracks the reference's.  Outputs are checked against the reference fixtures in
tests/test_oracle_golden.py; its time ratio to the real reference measured in the build
container is recorded in DESIGN.md.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sparse
import scipy.sparse.csgraph as csgraph
import scipy.sparse.linalg as spla
import torch

from .graphlearning_standin import _Graph, knn_exact


def sym_graph(data, k, epsilon, fast_knn=True):
    """Steps of knn_sym_dist (GLL.py:180-244): kNN, union-max, eps, W, V (+ modV, C)."""
    ind, dist = knn_exact(data, k, fast=fast_knn)
    n, kk = ind.shape
    owner = np.repeat(np.arange(n), kk)
    D = sparse.coo_matrix((dist.ravel(), (owner, ind.ravel())), shape=(n, n)).tocsr()
    DT = D.T
    D = D + DT.multiply(DT > D) - D.multiply(DT > D)                 # GLL.py:197
    r, c, v = sparse.find(D)                                         # GLL.py:198
    if epsilon == "auto":
        eps = D[ind[:, 0], [ind[:, -1]]].toarray().ravel()           # GLL.py:205
        Cd = np.zeros((n, n))                                        # GLL.py:209-213
        Cd[ind[:, -1], ind[:, 0]] = 1
        Cm = sparse.csr_matrix(Cd)
    else:
        eps = float(epsilon) * np.ones(n)
        Cm = 0
    scale = eps[r] * eps[c]
    Wv = np.exp(-4.0 * v * v / scale)
    Vv = -8.0 * Wv / scale
    W = sparse.coo_matrix((Wv, (r, c)), shape=(n, n)).tocsr()
    V = sparse.coo_matrix((Vv, (r, c)), shape=(n, n)).tocsr()
    modV = sparse.coo_matrix((v * v * Vv / eps[r] ** 2 / 2, (r, c)), shape=(n, n)).tocsr() \
        if epsilon == "auto" else 0
    return W, V, modV, Cm, ind


def forward(X: torch.Tensor, Y, tau=0.0, epsilon="auto", k=25):
    """Forward of GLL.py:14-73. Returns (U float64 tensor, saved dict)."""
    W, V, modV, Cm, ind = sym_graph(X.detach().cpu().numpy(), k, epsilon)
    L = csgraph.laplacian(W).tocsr()
    Yn = np.asarray(Y.detach().cpu().numpy() if torch.is_tensor(Y) else Y)
    base = Yn.shape[0]
    Luu = L[base:, base:]
    Lul = L[base:, :base]
    m = Luu.shape[0]
    Luu = Luu + sparse.spdiags(tau * np.ones(m), 0, m, m).tocsr()
    U = spla.spsolve(Luu, -Lul @ Yn)
    saved = dict(V=V, Luu=Luu, Y=Yn, modV=modV, C=Cm, X=X, U=U)
    return torch.from_numpy(np.asarray(U).reshape(m, -1)), saved


def backward(saved, gbar):
    """Backward of GLL.py:76-177. Returns grad_X (float32 tensor)."""
    X, U, Yn, V = saved["X"], saved["U"], saved["Y"], saved["V"]
    n = X.shape[0]
    g = gbar.detach().cpu().numpy() if torch.is_tensor(gbar) else np.asarray(gbar)
    w = spla.spsolve(saved["Luu"], g)
    w = np.concatenate((np.zeros_like(Yn), np.asarray(w).reshape(g.shape)), axis=0)
    P = np.concatenate((Yn, np.asarray(U).reshape(g.shape)), axis=0)
    graph = _Graph(-V)
    G = None
    for c in range(P.shape[1]):                                       # GLL.py:112-120
        term = graph.gradient(w[:, c]).transpose().multiply(graph.gradient(P[:, c]))
        G = term if G is None else G + term
    extra = 0
    if not isinstance(saved["C"], int):                               # GLL.py:124-139
        b = G.multiply(saved["modV"]).dot(np.ones(n))
        T = csgraph.laplacian(saved["C"].multiply(b), symmetrized=True)
        T = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((T.row, T.col))).long(),
                                    torch.from_numpy(T.data).float(), T.shape)
        extra = -(T @ X.detach())
    Gs = csgraph.laplacian(G.multiply(V))                             # GLL.py:146-159
    Gt = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((Gs.row, Gs.col))).long(),
                                 torch.from_numpy(Gs.data).float(), Gs.shape)
    return Gt @ X.detach() + extra
